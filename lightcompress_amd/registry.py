"""Name -> class registries (llmc/utils/registry_factory.py:1-49).

Algorithms register with ``@ALGO_REGISTRY`` exactly like the reference, so a YAML
``quant.method: GPTQ`` resolves to ``lightcompress_amd.gptq.GPTQ``.
"""


class Register(dict):
    def __init__(self, name):
        super().__init__()
        self.name = name

    def __call__(self, target):
        return self.register(target)

    def register(self, target, key=None):
        key = key or target.__name__
        if key in self:
            raise KeyError(f'{key} already registered in {self.name}')
        self[key] = target
        return target


ALGO_REGISTRY = Register('ALGO_REGISTRY')
MODEL_REGISTRY = Register('MODEL_REGISTRY')
