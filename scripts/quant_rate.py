"""Device rate of the grouped int quant kernels on Llama-3-8B linear shapes (GB/s at the
algorithmic bytes: input read + outputs written)."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from lightcompress_amd import ops  # noqa: E402

dev = torch.device('cuda:0')


def timed(fn, n=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


res = {}
w = (torch.randn(14336, 4096, device=dev) * 0.02).to(torch.bfloat16)
pre = (torch.rand(4096, device=dev) + 0.5).to(torch.bfloat16)
n = w.numel()
cases = {
    'fq_int4_asym_g128': (lambda: ops.int_quant_dynamic(w, 128, 0, 15, False, qparams=False), 4),
    'fq_int4_sym_g128_prescale': (lambda: ops.int_quant_dynamic(w, 128, -8, 7, True, pre_scale=pre,
                                                                qparams=False), 4),
    'pack_int4_asym_g128': (lambda: ops.int_quant_dynamic(w, 128, 0, 15, False, fq=False,
                                                          pack_bits=4), 2.5),
    'fq_int8_sym_perchannel': (lambda: ops.int_quant_dynamic(w, 0, -128, 127, True, qparams=False), 4),
}
for name, (fn, bpe) in cases.items():
    ms = timed(fn)
    res[name] = {'ms': round(ms, 4), 'GBps': round(n * bpe / ms / 1e6, 1)}
    print(name, res[name], flush=True)
print(json.dumps(res))
