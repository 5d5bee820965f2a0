"""World-size-2 gloo run of bench.py's data-parallel path on CPU.

Each rank runs the real SVDFormer PCN step on its own sample (point ops on
the oracle CPU path) under bench.wrap_ddp; the all-reduced gradients must be
identical on both ranks and equal the mean of the ranks' local gradients."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from bench import synth_pcn, wrap_ddp
    from oracle.cpu_path import cpu_ops, depth_images
    from svdformer_pointsea_amd.render import PCViews
    from svdformer_pointsea_amd.svdformer import Model, PCNConfig, get_loss

    torch.manual_seed(0)
    local = Model(PCNConfig)
    ddp = wrap_ddp(Model(PCNConfig), None)
    ddp.module.load_state_dict(local.state_dict())
    partial, gt = synth_pcn(1, 1000 + rank, "cpu")
    render = PCViews(TRANS=-0.7, RESOLUTION=224)
    with cpu_ops():
        depth = depth_images(render, partial).unsqueeze(1)
        for m in (local, ddp):
            loss, _ = get_loss(m(partial, depth), gt)
            loss.backward()
    names = [n for n, p in local.named_parameters() if p.grad is not None]
    g_local = torch.cat([dict(local.named_parameters())[n].grad.flatten() for n in names])
    g_ddp = torch.cat([dict(ddp.module.named_parameters())[n].grad.flatten() for n in names])
    mean_local = g_local.clone()
    dist.all_reduce(mean_local)
    mean_local /= world
    other = g_ddp.clone()
    dist.broadcast(other, src=0)
    out[rank] = (float((g_ddp - mean_local).abs().max()), float((g_ddp - other).abs().max()),
                 float(g_local.abs().max()))
    dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_ddp_gloo_world2():
    world = 2
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
        res = dict(out)
    for rank in range(world):
        diff_mean, diff_ranks, scale = res[rank]
        assert diff_ranks == 0.0
        assert diff_mean <= 1e-6 * max(scale, 1.0)
