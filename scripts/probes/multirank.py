"""Run the 2-rank-on-one-GPU rehearsal directly (debug aid): torchrun --nproc-per-node 2."""
import os, sys, traceback
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
sys.path.insert(0, str(Path(__file__).resolve().parents[2] / 'tests'))
import torch, torch.distributed as dist
import test_multirank_gpu as T
rank = int(os.environ['RANK'])
torch.cuda.set_device(0)
dist.init_process_group('gloo')
which = sys.argv[1]
cfg, layers = {'awq': (T.AWQ, 4), 'gptq': (T.GPTQ, 2)}[which]
try:
    out = T._run(cfg, layers)
    print(rank, 'ok', len(out), flush=True)
except Exception:
    traceback.print_exc()
    raise
finally:
    dist.destroy_process_group()
