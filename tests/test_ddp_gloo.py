"""World-size-2 gloo run of bench.py's data-parallel path on CPU.

Each rank runs the real SVDFormer PCN step on its own sample (point ops on
the oracle CPU path) with train.FlatParams (bench.py's parameter storage):
gradients accumulate into one flat buffer whose all-reduce is the step's
only collective -- issued once after backward, or bucket by bucket from
backward hooks (train.BucketedAllReduce, bitwise the same).  After it, the
gradients must be identical on both ranks and equal the mean of the ranks'
local gradients, and one Adam step must leave identical weights."""
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
    from bench import synth_pcn
    from svdformer_pointsea_amd.train import FlatParams
    from oracle.cpu_path import cpu_ops, depth_images
    from svdformer_pointsea_amd.render import PCViews
    from svdformer_pointsea_amd.svdformer import Model, PCNConfig, get_loss

    torch.manual_seed(0)
    model = Model(PCNConfig)
    fp = FlatParams(model, "cpu", bf16=False)
    partial, gt = synth_pcn(1, 1000 + rank, "cpu")
    render = PCViews(TRANS=-0.7, RESOLUTION=224)
    with cpu_ops():
        depth = depth_images(render, partial).unsqueeze(1)
        fp.zero_grad()
        loss, _ = get_loss(fp.forward(partial, depth), gt)
        loss.backward()
        fp.collect()
    local = fp.grad.clone()
    # the overlapped path: the same step with bucketed all-reduces issued from
    # backward hooks (small buckets -> many collectives) must give the single
    # all-reduce's gradients bitwise
    from svdformer_pointsea_amd.train import BucketedAllReduce

    sync = BucketedAllReduce(fp, world, bucket_mb=4.0)
    with cpu_ops():
        fp.zero_grad()
        loss, _ = get_loss(fp.forward(partial, depth), gt)
        loss.backward()
        sync.finish()
    bucketed = fp.grad.clone()
    for h in sync._hooks:
        h.remove()
    fp.grad.copy_(local)
    fp.allreduce(world)
    n_buckets = len(sync.buckets)
    mean_local = local.clone()
    dist.all_reduce(mean_local)
    mean_local /= world
    other = fp.grad.clone()
    dist.broadcast(other, src=0)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    opt.step()
    w = torch.cat([p.detach().flatten() for p in model.parameters()])
    w0 = w.clone()
    dist.broadcast(w0, src=0)
    out[rank] = (float((fp.grad - mean_local).abs().max()), float((fp.grad - other).abs().max()),
                 float(local.abs().max()), float((w - w0).abs().max()),
                 bool(torch.equal(bucketed[:fp.n_train], fp.grad[:fp.n_train])), n_buckets)
    dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_ddp_gloo_world2():
    world = 2
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
        res = dict(out)
    for rank in range(world):
        diff_mean, diff_ranks, scale, diff_w, bucketed_equal, n_buckets = res[rank]
        assert diff_ranks == 0.0 and diff_w == 0.0
        assert bucketed_equal and n_buckets > 5
        assert diff_mean <= 1e-6 * max(scale, 1.0)
