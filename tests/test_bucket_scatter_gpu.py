"""mhppo_bucket_scatter (bucket_segments' segment-major cross/wait buckets in one pass)
against index_select of the same time-major buffers: bit-exact, for random disjoint
segment sets (ragged NS and T against the kernel's 64-segment x 16-step blocks), an empty
bucket, both buckets empty, and a single segment."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("T,NS,p0,p1", [(80, 4099, 0.4, 0.4), (80, 262144, 0.45, 0.45), (7, 1, 1.0, 0.0),
                                        (80, 20000, 0.0, 0.5), (33, 130, 0.0, 0.0)])
def test_bucket_scatter_matches_index_select(T, NS, p0, p1):
    from mhppo.rollout import scatter_buckets
    g = torch.Generator().manual_seed(T * NS)
    obs = torch.randn(T, NS, 13, generator=g).cuda()
    act, logp, ret = (torch.randn(T, NS, generator=g).cuda() for _ in range(3))
    rew = torch.randn(T, NS, generator=g, dtype=torch.float64).cuda()
    u = torch.rand(NS, generator=g)
    segs = [torch.nonzero(u < p0).squeeze(1).cuda(), torch.nonzero((u >= p0) & (u < p0 + p1)).squeeze(1).cuda()]
    outs = scatter_buckets(segs[0], segs[1], NS, T, obs, act, logp, ret, rew)
    torch.cuda.synchronize()
    for seg, o in zip(segs, outs):
        idx = (seg.unsqueeze(1) + torch.arange(T, device="cuda") * NS).reshape(-1)
        assert o["n_seg"] == seg.numel()
        assert torch.equal(o["obs"], obs.reshape(-1, 13).index_select(0, idx))
        for k, x in (("act", act), ("logp", logp), ("ret", ret), ("rew", rew)):
            assert torch.equal(o[k], x.reshape(-1).index_select(0, idx)), k
