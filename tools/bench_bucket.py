"""Time mhppo_bucket_scatter at the bench's shape (config 3: NS = 65 536 envs x 4 slots
segments, T = 80 steps, ~half the segments in each bucket) with HIP events on the launch
stream.  MHPPO_LIB selects the library build (A/B).  Prints ms per launch and the HBM rate
over the algorithmic bytes (72 B read + 72 B written per bucketed record)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mh-ppo_amd")]
import torch  # noqa: E402
from mhppo import _lib  # noqa: E402

NS, T, NF = int(os.environ.get("NS", 262144)), 80, 13
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(1)
obs = torch.randn(T, NS, NF, device=dev, generator=g)
act, logp, ret = (torch.randn(T, NS, device=dev, generator=g) for _ in range(3))
rew = torch.randn(T, NS, device=dev, dtype=torch.float64, generator=g)
u = torch.rand(NS, device=dev, generator=g)
# EXIST < 1: that fraction of segments exists (the scalable env's ragged slots); the rest are in
# neither bucket (pos = -1) and must not be fetched
ex = torch.rand(NS, device=dev, generator=g) < float(os.environ.get("EXIST", "1"))
segs = [torch.nonzero((u < 0.5) & ex).squeeze(1), torch.nonzero((u >= 0.5) & ex).squeeze(1)]
pos = torch.full((NS,), -1, dtype=torch.int64, device=dev)
bucket = torch.zeros(NS, dtype=torch.int8, device=dev)
dst, keep = (_lib.BucketDst * 2)(), []
for b, seg in enumerate(segs):
    n = seg.numel()
    pos[seg] = torch.arange(n, dtype=torch.int64, device=dev)
    bucket[seg] = b
    o = [torch.empty(n * T, NF, device=dev)] + [torch.empty(n * T, device=dev) for _ in range(3)] + \
        [torch.empty(n * T, device=dev, dtype=torch.float64)]
    keep.append(o)
    dst[b] = _lib.BucketDst(*[x.data_ptr() for x in o])
L = _lib.lib()
args = [_lib.ptr(pos), _lib.ptr(bucket), NS, T] + [_lib.ptr(x) for x in (obs, act, logp, ret, rew)] + [dst]


def run(k):
    s = _lib.stream_ptr(device=dev)
    for _ in range(k):
        _lib.check(L.mhppo_bucket_scatter(*args, s))


run(3)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
K = 50
e0.record()
run(K)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / K
nrec = T * NS
byts = 144 * T * sum(s.numel() for s in segs)  # bucketed records: read + written
print(f"{os.environ.get('TAG', 'lib')}: bucket_scatter {ms * 1e3:.1f} us  {byts / ms / 1e6:.0f} GB/s "
      f"({byts / 1e9:.3f} GB algorithmic)")
