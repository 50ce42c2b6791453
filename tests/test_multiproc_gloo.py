"""World-size-2 gloo tests of the N > 1 path on CPU (no GPU needed).

What a multi-GPU run relies on besides the device code:
- every rank builds the SAME full scene (bench.py generates it per rank from
  the seed; the library then partitions it), checked by hashing on each rank;
- the frame partition every shard computes (mmba_shard_layout, the code
  Plan::build uses) is identical on all ranks, covers the frames contiguously,
  gives every observation and every bundle exactly one owner and balances
  observations;
- bench.py's torch.distributed plumbing: the 128-byte RCCL id broadcast, the
  barrier and the max-over-ranks timing.
"""
import hashlib
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _problem_digest(p):
    h = hashlib.sha256()
    for name in ("attr_values", "obs_xy", "obs_weight", "obs_frame", "obs_marker", "mkr_bnd",
                 "mkr_cam", "param_attr", "param_frame"):
        if hasattr(p, name):
            h.update(np.ascontiguousarray(getattr(p, name)).tobytes())
    return h.hexdigest()


def _worker(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["RANK"] = str(rank)
    os.environ["WORLD_SIZE"] = str(world)
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    import bench
    from mayamatchmovesolver_amd import synthetic as S
    from mayamatchmovesolver_amd.solver import shard_layout

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # weak scaling as bench.py does it: the per-rank shard is a fixed
        # frame count, the scene has world x that many frames
        frames = 24 * world
        prob = S.make_config(3, frames=frames, scale=0.01 * world)
        dig = _problem_digest(prob)
        digs = [None] * world
        dist.all_gather_object(digs, dig)
        assert len(set(digs)) == 1, "ranks built different scenes"

        bounds, owner = shard_layout(prob, world)
        allb = [None] * world
        dist.all_gather_object(allb, (bounds.tolist(), owner.tolist()))
        assert all(b == allb[0] for b in allb), "ranks disagree on the partition"

        # RCCL id broadcast and timing reduction exactly as bench.py does them
        uid = bytes(range(128)) if rank == 0 else None
        got = bench.broadcast_bytes(dist, uid, 128)
        assert got == bytes(range(128))
        bench.barrier(dist)
        assert bench.allreduce(dist, float(rank + 1), "max") == float(world)
        assert bench.allreduce(dist, 1.0, "sum") == float(world)

        np.savez(os.path.join(outdir, "rank%d.npz" % rank), bounds=bounds, owner=owner,
                 frames=np.asarray(prob.obs_frame),
                 bnd=np.asarray(prob.mkr_bnd)[np.asarray(prob.obs_marker)])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_sharded_layout(tmp_path, world):
    import torch.multiprocessing as mp

    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r = [np.load(tmp_path / ("rank%d.npz" % k)) for k in range(world)]
    bounds, owner, frames, bnd = r[0]["bounds"], r[0]["owner"], r[0]["frames"], r[0]["bnd"]
    F = int(frames.max()) + 1
    # contiguous cover of the frames
    assert bounds[0] == 0 and bounds[-1] == F
    assert np.all(np.diff(bounds) > 0)
    # every observation owned by exactly one shard, counts balanced to within
    # one frame's observations
    shard_of_obs = np.searchsorted(bounds, frames, side="right") - 1
    counts = np.bincount(shard_of_obs, minlength=world)
    assert counts.sum() == frames.size
    per_frame = np.bincount(frames, minlength=F)
    assert counts.max() - counts.min() <= 2 * per_frame.max()
    # a bundle belongs to the shard of its earliest observation
    first = np.full(owner.size, F)
    np.minimum.at(first, bnd, frames)
    seen = first < F
    expect = np.searchsorted(bounds, first[seen], side="right") - 1
    assert np.array_equal(owner[seen], expect)
