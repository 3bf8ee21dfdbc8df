"""Two ranks on the GPU box (both on cuda:0, gloo transport) running the HIP training step
under ArenaDataParallel, checked against the reference's 2-rank DDP golden
(oracle/make_goldens.py capture_ddp: strided batch[rank::2] sharding, trainer.py:604-619
loss weighting, DDP gradient averaging, rank-local BatchNorm statistics)."""
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _worker(rank, world, init, q):
    import sys
    import os
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.join(os.path.dirname(here), "espnet-1_amd")]
    from goldens import load, section
    from test_model_build import build
    from espnet_amd.train.distributed import ArenaDataParallel

    dist.init_process_group("gloo", init_method=f"file://{init}", rank=rank, world_size=world)
    meta, d = load("ddp2")
    cfg, g0 = load(meta["cfg_name"])
    torch.manual_seed(0)
    m = build(cfg)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in section(g0, "w").items()})
    m.prepare("cuda:0", amp=False)
    m.train()
    dp = ArenaDataParallel(m, bucket_mb=0.25)
    full = {k: torch.from_numpy(v) for k, v in section(d, "in").items()}
    batch = {k: v[rank::world] for k, v in full.items()}
    dp.broadcast_buffers()
    loss, stats, weight = m(**batch)
    stats = {k: v for k, v in stats.items() if v is not None}
    loss, stats, weight = dp.weighted_average(loss, stats, weight)
    dp.begin_backward()
    loss.backward()
    dp.allreduce_grads()
    torch.cuda.synchronize()
    if rank == 0:
        out = dict(loss=float(loss.detach()) * world, weight=int(weight),
                   stats={k: float(v) for k, v in stats.items()},
                   grads={k: p.grad.cpu().numpy() for k, p in m.named_parameters()},
                   bufs={k: v.cpu().numpy() for k, v in m.state_dict().items() if "running" in k or "num_batches" in k})
        q.put(out)
    dist.barrier()
    dist.destroy_process_group()


def test_ddp_two_ranks_matches_reference_golden():
    from goldens import load, section
    _, d = load("ddp2")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = tempfile.mktemp(prefix="ea_ddp_gpu_")
    ps = [ctx.Process(target=_worker, args=(r, 2, init, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = q.get(timeout=140)
    for p in ps:
        p.join(120)
    np.testing.assert_allclose(out["loss"], d["out.loss_scaled"], rtol=2e-6, atol=1e-4)
    assert out["weight"] == int(d["out.weight"])
    for k, v in section(d, "stat").items():
        np.testing.assert_allclose(out["stats"][k], v, rtol=2e-6, atol=1e-4, err_msg=k)
    for k, g in section(d, "g").items():
        np.testing.assert_allclose(out["grads"][k], g, atol=2e-5, rtol=2e-4, err_msg=k)
    for k, v in section(d, "buf_after").items():
        np.testing.assert_allclose(out["bufs"][k], v, atol=1e-5, rtol=1e-5, err_msg=k)
