"""CPU, world_size 2 over gloo: the multi-GPU sharding and collectives are exact.

The per-shard renderer is the CPU oracle here (the HIP renderer plugs into the same slot on the
GPU box); what is under test is the chunk-aligned split, the ragged all-gather and frame
ordering: the sharded result must be bit-identical to the single-process one.
"""
import importlib
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    sys.path.insert(0, REPO)
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from _golden import Golden
        D = importlib.import_module("a-nerf_amd.distributed")
        g = Golden("h1_nanfill_s32i16_d4w128")
        om = oracle.OracleModel(g.cfg, g.ckpt)
        rb = torch.from_numpy(np.concatenate([g.ray_batch()] * 3)[:9000])  # 3 chunks of 4096 (ragged last)

        def render_fn(sl):
            o = om.render_rays(sl.numpy(), g["skts"][0], g["cyls"][0:1], chunk=4096)
            return {k: torch.from_numpy(v) for k, v in o.items()}

        out = D.render_rays_sharded(render_fn, rb, chunk=4096)
        # the static-size gather bench.py uses (one all_gather_into_tensor, padding dropped)
        s0, s1 = D.chunk_ranges(rb.shape[0], 4096, world)[rank]
        sg = D.ShardGather(rb.shape[0], 4096, world, torch.device("cpu"))(render_fn(rb[s0:s1]))
        for k in out:
            assert torch.equal(sg[k], out[k]), k

        # ray-balanced ranges (rank 1 starts mid-chunk): near / far filled over the covering chunks
        def near_far_fn(rays):
            near, far, _, _ = om.near_far(rays.numpy(), g["cyls"][0:1], chunk=4096)
            return torch.from_numpy(near), torch.from_numpy(far)

        def render_nf(sl, near, far):
            o = om.render_rays(sl.numpy(), g["skts"][0], g["cyls"][0:1], chunk=4096, near=near.numpy(),
                               far=far.numpy())
            return {k: torch.from_numpy(v) for k, v in o.items()}
        outb = D.render_rays_sharded(render_nf, rb, chunk=4096, near_far_fn=near_far_fn)
        r0, r1 = D.ray_ranges(rb.shape[0], world)[rank]
        c0, c1 = D.chunk_cover(r0, r1, 4096, rb.shape[0])
        nf = near_far_fn(rb[c0:c1])
        sgb = D.ShardGather(rb.shape[0], 4096, world, torch.device("cpu"), ranges=D.ray_ranges(rb.shape[0], world))(
            render_nf(rb[r0:r1], nf[0][r0 - c0:r1 - c0], nf[1][r0 - c0:r1 - c0]))
        for k in out:
            assert torch.equal(outb[k], out[k]) and torch.equal(sgb[k], out[k]), k
        # tiles dealt round-robin (what bench.py runs): near / far over the whole list, this rank's tiles
        outt = D.render_rays_sharded(render_nf, rb, chunk=4096, near_far_fn=near_far_fn, split="tiles", tile=1000)
        rows = [D.tile_rows(rb.shape[0], world, r, 1000) for r in range(world)]
        nfa = near_far_fn(rb)
        mine_r = rows[rank]
        sgt = D.ShardGather(rb.shape[0], 4096, world, torch.device("cpu"), rank_rows=rows)(
            render_nf(rb[mine_r], nfa[0][mine_r], nfa[1][mine_r]))
        for k in out:
            assert torch.equal(outt[k], out[k]) and torch.equal(sgt[k], out[k]), k
        frames = torch.arange(5 * 4 * 4 * 3, dtype=torch.float32).reshape(5, 4, 4, 3)
        mine = frames[D.frame_ids(5, rank, world)]
        full = D.gather_frames(mine, 5)
        if rank == 0:
            q.put(({k: v.numpy() for k, v in out.items()}, torch.equal(full, frames)))
    finally:
        dist.destroy_process_group()


def test_chunk_ranges_are_whole_chunks_and_cover():
    D = importlib.import_module("a-nerf_amd.distributed")
    for n in (0, 1, 4095, 4096, 4097, 213598):
        for w in (1, 2, 3, 8):
            rs = D.chunk_ranges(n, 4096, w)
            assert rs[0][0] == 0 and rs[-1][1] == n
            for (a, b), (c, _) in zip(rs, rs[1:]):
                assert b == c and a % 4096 == 0
    assert D.frame_ids(5, 1, 2) == [1, 3]
    for n in (0, 1, 9000, 853182):
        for w in (1, 2, 3, 8):
            rs = D.ray_ranges(n, w)
            assert rs[0][0] == 0 and rs[-1][1] == n and max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1
            for (a, b), (c, _) in zip(rs, rs[1:]):
                assert b == c
            for a, b in rs:
                c0, c1 = D.chunk_cover(a, b, 4096, n)
                assert c0 % 4096 == 0 and (c1 % 4096 == 0 or c1 == n) and c0 <= a and b <= c1
            for tile in (1, 256, 1000):
                rows = [D.tile_rows(n, w, r, tile) for r in range(w)]
                allr = torch.cat(rows)
                assert allr.shape[0] == n and torch.equal(torch.sort(allr).values, torch.arange(n))
                sizes = [int(r.shape[0]) for r in rows]
                assert max(sizes) - min(sizes) <= tile


@pytest.mark.timeout(600)
def test_gloo_world2_sharded_render_is_bit_identical():
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    from _golden import Golden
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res, frames_ok = q.get(timeout=600)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    g = Golden("h1_nanfill_s32i16_d4w128")
    rb = np.concatenate([g.ray_batch()] * 3)[:9000]
    ref = oracle.OracleModel(g.cfg, g.ckpt).render_rays(rb, g["skts"][0], g["cyls"][0:1], chunk=4096)
    for k in ("rgb_map", "disp_map", "acc_map"):
        np.testing.assert_array_equal(res[k], ref[k])
    assert frames_ok
