"""Multi-GPU rendering: one process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI).

The reference's only parallelism is nn.DataParallel (core/raycasters.py:157, run_render.py:111):
every forward re-broadcasts the weights, scatters a 4096-ray chunk over the GPUs and gathers
the outputs on GPU 0 — and its chunk-coupled NaN fill then depends on the GPU count.  Here:

* weights are uploaded once per rank (anerf_model_create), never re-broadcast;
* `pixels` mode (the north star's layout, BASELINE config 5; what bench.py runs under the launcher
  at every N): one frame's bounding-box ray list is split over the ranks, each rank renders its
  rays, and one all-gather of (rgb, disp, acc) assembles the ray outputs on every rank before
  composition.  Three splits:
  `tiles` (default) — 256-ray tiles dealt round-robin over the ranks (tile_rows).  Per-ray cost is
  not constant (exact-zero cutoff-window skipping: a ray costs what its live joints cost), and
  contiguous bands concentrate the torso's rays: measured on one GPU over config 5's 1024^2 frame
  (tools/shard_balance.py, profiles/r04a_shard_balance.jsonl), the slowest of 8 equal-ray
  contiguous ranges took 1.051x the mean, the slowest of 8 tile sets 1.002x.  Every rank fills
  near / far over the whole frame's chunks (0.1 ms) and renders its tiles with them
  (ANERF_FLAG_NEAR_FAR);
  `rays` — contiguous equal-ray ranges (ray_ranges), near / far over the chunks covering the range
  (chunk_cover);
  `chunks` — ranges of whole `chunk`-ray chunks (chunk_ranges), so each rank's own NaN fill is the
  single-GPU one.
  Results are bit-identical to the single-GPU render with every split;
* `frames` mode (throughput over many frames): frames are independent, rank r renders frames
  r, r+N, ... with no collective in the data path; `gather_frames` optionally all-gathers them.
The render function is injectable (default: the HIP RayCaster) so the sharding and collective
logic is tested with gloo on CPU.
"""
import torch
import torch.distributed as dist


def chunk_ranges(n_rays, chunk, world):
    """Contiguous [start, stop) ray ranges made of whole chunks, balanced by chunk count."""
    n_chunks = (n_rays + chunk - 1) // chunk
    out = []
    for r in range(world):
        c0 = (r * n_chunks) // world
        c1 = ((r + 1) * n_chunks) // world
        out.append((min(c0 * chunk, n_rays), min(c1 * chunk, n_rays)))
    return out


def ray_ranges(n_rays, world):
    """Contiguous [start, stop) ray ranges balanced by ray count."""
    return [((r * n_rays) // world, ((r + 1) * n_rays) // world) for r in range(world)]


def tile_rows(n_rays, world, rank, tile=256):
    """Ray indices of `rank` when the ray list is cut into `tile`-ray tiles dealt round-robin over the
    ranks (tile t -> rank t % world): every rank gets rows from the whole frame, so the per-ray cost's
    spatial variation (live joints) averages out.  Returns an int64 CPU tensor, ascending."""
    n_tiles = (n_rays + tile - 1) // tile
    if rank >= n_tiles:
        return torch.zeros(0, dtype=torch.int64)
    t = torch.arange(rank, n_tiles, world, dtype=torch.int64)
    rows = (t[:, None] * tile + torch.arange(tile, dtype=torch.int64)[None, :]).reshape(-1)
    return rows[rows < n_rays]


def chunk_cover(s0, s1, chunk, n_rays):
    """The whole-chunk range [c0, c1) that contains rays [s0, s1) (the rays whose NaN fill they share)."""
    if s1 <= s0:
        return s0, s0
    return (s0 // chunk) * chunk, min(((s1 + chunk - 1) // chunk) * chunk, n_rays)


def frame_ids(n_frames, rank, world):
    return list(range(rank, n_frames, world))


def all_gather_rows(t, group=None):
    """all_gather of a [n_local, ...] tensor with ragged n_local: pad to the max, gather, trim."""
    world = dist.get_world_size(group)
    n = torch.tensor([t.shape[0]], device=t.device, dtype=torch.int64)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    m = max(sizes)
    pad = torch.zeros((m,) + tuple(t.shape[1:]), device=t.device, dtype=t.dtype)
    pad[: t.shape[0]] = t
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad, group=group)
    return torch.cat([b[:s] for b, s in zip(bufs, sizes)], 0)


def render_rays_sharded(render_fn, ray_batch, chunk, group=None, near_far_fn=None, split=None, tile=256):
    """Pixel sharding of one ray list, then one all-gather of [rgb(3), disp, acc] per ray.
    Without near_far_fn: rank r renders its whole-chunk range, render_fn(ray_slice) ->
    dict(rgb_map, disp_map, acc_map).  With near_far_fn(rays) -> (near, far) (the chunk NaN fill over
    the given rays, e.g. raycaster.near_far) and split "tiles" (the default then): the rank fills
    near / far over the whole list and calls render_fn(its_tile_rays, near, far); split "rays":
    ray-balanced contiguous ranges, near / far over the chunks covering the range."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    n = ray_batch.shape[0]
    split = split or ("chunks" if near_far_fn is None else "tiles")
    rows = None
    if split == "chunks":
        s0, s1 = chunk_ranges(n, chunk, world)[rank]
    elif split == "rays":
        s0, s1 = ray_ranges(n, world)[rank]
    elif split == "tiles":
        rows = tile_rows(n, world, rank, tile).to(ray_batch.device)
    else:
        raise ValueError(f"split {split!r}: 'tiles', 'rays' or 'chunks'")
    if split != "chunks" and near_far_fn is None:
        raise ValueError(f"split {split!r} needs near_far_fn (the chunk NaN fill over other ranks' rays)")
    m = rows.shape[0] if rows is not None else s1 - s0
    if m > 0:
        if split == "chunks":
            out = render_fn(ray_batch[s0:s1])
        elif split == "rays":
            c0, c1 = chunk_cover(s0, s1, chunk, n)
            near, far = near_far_fn(ray_batch[c0:c1])
            out = render_fn(ray_batch[s0:s1], near[s0 - c0:s1 - c0], far[s0 - c0:s1 - c0])
        else:
            near, far = near_far_fn(ray_batch)
            out = render_fn(ray_batch.index_select(0, rows), near.index_select(0, rows), far.index_select(0, rows))
        local = torch.cat([out["rgb_map"].reshape(-1, 3), out["disp_map"].reshape(-1, 1),
                           out["acc_map"].reshape(-1, 1)], -1).contiguous()
    else:
        local = torch.zeros(0, 5, device=ray_batch.device, dtype=torch.float32)
    full = all_gather_rows(local, group)
    if split != "tiles":
        return {"rgb_map": full[:, 0:3], "disp_map": full[:, 3], "acc_map": full[:, 4]}
    order = torch.cat([tile_rows(n, world, r, tile) for r in range(world)]).to(full.device)
    frame = torch.empty_like(full)
    frame[order] = full
    return {"rgb_map": frame[:, 0:3], "disp_map": frame[:, 3], "acc_map": frame[:, 4]}


class ShardGather:
    """The all-gather of render_rays_sharded with its sizes fixed up front (chunk_ranges is known on
    every rank): per call ONE all_gather_into_tensor of a [world * m, 5] buffer (m = the largest
    range) and one row gather that drops the padding — no size exchange, no host sync.
    `ranges`: the ranks' [start, stop) (default chunk_ranges; ray_ranges for ray-balanced sharding),
    or `rank_rows`: each rank's ray indices (tile_rows for the tiled split), any disjoint cover.
    __call__(out) -> dict(rgb_map, disp_map, acc_map) of the whole ray list, ray order."""

    def __init__(self, n_rays, chunk, world, device, group=None, ranges=None, rank_rows=None):
        if rank_rows is None:
            self.ranges = ranges if ranges is not None else chunk_ranges(n_rays, chunk, world)
            rank_rows = [torch.arange(s0, s1) for s0, s1 in self.ranges]
        rank_rows = [torch.as_tensor(r, dtype=torch.int64).cpu() for r in rank_rows]
        assert len(rank_rows) == world
        self.m = max(max(int(r.shape[0]) for r in rank_rows), 1)
        self.group = group
        # frame row i comes from gathered row src[i] (rank r's k-th ray sits at r * m + k)
        src = torch.full((n_rays,), -1, dtype=torch.int64)
        for r, rows in enumerate(rank_rows):
            src[rows] = r * self.m + torch.arange(rows.shape[0])
        assert bool((src >= 0).all()), "rank_rows must cover every ray"
        self.rows = src.to(device)
        self.local = torch.zeros(self.m, 5, device=device, dtype=torch.float32)
        self.full = torch.empty(world * self.m, 5, device=device, dtype=torch.float32)

    def __call__(self, out):
        if out is not None:
            k = out["rgb_map"].shape[0]
            self.local[:k, 0:3] = out["rgb_map"].reshape(-1, 3)
            self.local[:k, 3] = out["disp_map"].reshape(-1)
            self.local[:k, 4] = out["acc_map"].reshape(-1)
        dist.all_gather_into_tensor(self.full, self.local, group=self.group)
        g = self.full.index_select(0, self.rows)
        return {"rgb_map": g[:, 0:3].contiguous(), "disp_map": g[:, 3].contiguous(), "acc_map": g[:, 4].contiguous()}


def gather_frames(local_frames, n_frames, group=None):
    """All-gather per-rank frames ([F_local, H, W, C] tensors) back into frame order."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    g = all_gather_rows(local_frames, group)
    order = [f for r in range(world) for f in frame_ids(n_frames, r, world)]
    out = torch.empty_like(g)
    out[torch.tensor(order, device=g.device)] = g
    return out
