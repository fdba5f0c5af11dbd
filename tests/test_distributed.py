"""Multi-rank partition and framebuffer gather on CPU (gloo, world_size 2).

The GPU render of each rank's tiles is stood in for by packing the oracle's
image into the tile-packed slab layout (no GPU here; the packed kernel output
is checked against the same layout on the GPU in test_gpu_parity.py); what is
under test is the product's tile ownership (raytracer_amd.distributed) and
the slab gather to rank 0 (gather_slabs), the same code bench.py runs over
RCCL, plus bench.py's multi-process launcher.
"""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("W,H,world", [(37, 21, 2), (64, 64, 3), (8, 9, 4), (800, 800, 8)])
def test_owner_masks_partition_the_image(W, H, world):
    from raytracer_amd.distributed import owner_mask
    cover = sum(owner_mask(W, H, (0, 0, W, H), r, world).astype(int) for r in range(world))
    assert cover.min() == 1 and cover.max() == 1
    # a sub-region partition covers exactly the region
    cover = sum(owner_mask(W, H, (3, 2, W - 5, H - 3), r, world).astype(int) for r in range(world))
    assert cover[2:H - 1, 3:W - 2].min() == 1 and cover.sum() == (W - 5) * (H - 3)


def pack_np(img, region, rank, world):
    """Restatement of the kernels' packed output: owned tile k, lane l -> k*64 + l."""
    from raytracer_amd import distributed as rtd
    H, W = img.shape[:2]
    x, y, w, h = rtd.clamp_region(region, W, H)
    tiles_x = -(-w // 8)
    slab = np.zeros((rtd.slab_tiles((x, y, w, h), world) * 64, *img.shape[2:]), img.dtype)
    for k, t in enumerate(rtd.owned_tiles((x, y, w, h), rank, world)):
        ty, tx = divmod(t, tiles_x)
        for l in range(64):
            i, j = x + tx * 8 + l % 8, y + ty * 8 + l // 8
            if i < x + w and j < y + h:
                slab[k * 64 + l] = img[j, i]
    return slab


def unpack_np(slabs, region, W, H, frame):
    """Restatement of rt_tiles_unpack (frame.hip)."""
    from raytracer_amd import distributed as rtd
    x, y, w, h = rtd.clamp_region(region, W, H)
    world = slabs.shape[0]
    for r in range(world):
        tiles_x = -(-w // 8)
        for k, t in enumerate(rtd.owned_tiles((x, y, w, h), r, world)):
            ty, tx = divmod(t, tiles_x)
            for l in range(64):
                i, j = x + tx * 8 + l % 8, y + ty * 8 + l // 8
                if i < x + w and j < y + h:
                    frame[j, i] = slabs[r, k * 64 + l]
    return frame


def test_pack_unpack_roundtrip():
    rng = np.random.default_rng(1)
    img = rng.integers(0, 255, (21, 37, 3), dtype=np.uint8)
    for world in (1, 2, 3, 5):
        for region in [(0, 0, 37, 21), (3, 2, 30, 40)]:
            slabs = np.stack([pack_np(img, region, r, world) for r in range(world)])
            out = unpack_np(slabs, region, 37, 21, np.zeros_like(img))
            from raytracer_amd.distributed import clamp_region
            x, y, w, h = clamp_region(region, 37, 21)
            assert np.array_equal(out[y:y + h, x:x + w], img[y:y + h, x:x + w])
            assert out.sum() == img[y:y + h, x:x + w].sum()


def _worker(rank, world, port, full_rgb, full_rad, q):
    import torch
    import torch.distributed as dist
    from raytracer_amd.distributed import gather_slabs, slab_tiles
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    H, W = full_rgb.shape[:2]
    region = (0, 0, W, H)
    slab = torch.from_numpy(pack_np(full_rgb, region, rank, world))
    rslab = torch.from_numpy(pack_np(full_rad, region, rank, world))
    assert slab.shape[0] == slab_tiles(region, world) * 64
    g = gather_slabs(slab, world)
    gr = gather_slabs(rslab, world)
    if rank == 0:
        rgb = unpack_np(g.numpy(), region, W, H, np.zeros_like(full_rgb))
        rad = unpack_np(gr.numpy(), region, W, H, np.zeros_like(full_rad))
        q.put((rgb, rad, int(slab.numel())))
    else:
        assert g is None
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_two_rank_gather_equals_full_render(oracle, rt):
    import torch.multiprocessing as mp
    sd = rt.generate_scene_data({"type": "cornell"})
    full = oracle.render(sd, {"width": 40, "samples": 4, "depth": 6, "aTolerance": 0})
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, full["rgb"], full["radiance"], q)) for r in range(2)]
    for p in procs:
        p.start()
    rgb, rad, slab_elems = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(rgb, full["rgb"])
    assert np.array_equal(rad, full["radiance"])
    assert slab_elems == 13 * 64 * 3  # 25 tiles over 2 ranks: frame/world (+ padding), not a full frame


def _bench(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True,
                          env=env, timeout=timeout, cwd=str(ROOT))


def test_bench_launcher_spawns_world_two():
    """bench.py --gpus 2 (no torch.distributed.run env): starts 2 ranks as a child
    process and forwards rank 0's line; the ranks really gathered (gloo stub)."""
    r = _bench(["--gpus", "2", "--stub", "--width", "37", "--steps", "1", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    assert lines[0]["n_gpus"] == 2 and lines[0]["stub_frame_ok"] is True
    assert lines[0]["slab_bytes_per_rank"] < lines[0]["frame_bytes"]


def test_bench_world_size_mismatch_fails():
    r = _bench(["--gpus", "4", "--stub"], env_extra={"WORLD_SIZE": "2"})
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_bench_metric_names_the_workload():
    import bench
    assert bench.metric_for("cornell", 800, 800, 256, 16) == bench.HEADLINE_METRIC
    m = bench.metric_for("spheres100k", 4096, 4096, 1024, 100)
    assert "spheres-100k" in m and "4096×4096" in m and "spp=1024" in m


def _words_of(st):
    """The 8 stats words (rt_camera_stats_words layout) of an oracle render's stats."""
    none = -1  # ~0 as int64
    s, b = st["samples"], st["bounces"]
    return [int(st["pixels"]), int(s["total"]), none if s["min"] == float("inf") else int(s["min"]), int(s["max"]),
            int(b["total"]), none if b["min"] == float("inf") else int(b["min"]), int(b["max"]), 0]


def _stats_worker(rank, world, port, words, n_px, q):
    import torch
    import torch.distributed as dist
    from raytracer_amd.distributed import gather_slabs, gathered_stats, stats_from_words
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # a u8 slab with the spare tile: pixels (here zeros), then the stats words
    slab = torch.zeros((n_px + 64, 3), dtype=torch.uint8)
    slab.view(-1)[n_px * 3:n_px * 3 + 64].view(torch.int64).copy_(torch.tensor(words[rank], dtype=torch.int64))
    g = gather_slabs(slab, world)
    if rank == 0:
        st = stats_from_words(gathered_stats(g, n_px).tolist())
        q.put((st.pixels, st.samples, st.bounces))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_two_rank_stats_merge_equals_single_render(oracle, rt):
    """RenderStats across ranks (RenderStats.merge, src/render-utils/renderStats.ts:
    42-64): each rank's 8 stats words ride in its slab's spare tile through the
    gather; rank 0's merge equals the stats of one render of the whole region.
    Adaptive sampling makes min / max per-pixel sample counts differ by rank."""
    import torch.multiprocessing as mp
    sd = rt.generate_scene_data({"type": "cornell"})
    ro = {"width": 24, "samples": 30, "depth": 6, "aTolerance": 0.05, "aBatch": 10}
    full = oracle.render(sd, ro)
    W, H = full["width"], full["height"]
    parts = [oracle.render(sd, ro, region=(0, 0, W, H // 3)), oracle.render(sd, ro, region=(0, H // 3, W, H - H // 3))]
    words = [_words_of(p["stats"]) for p in parts]
    assert parts[0]["stats"]["samples"]["total"] != parts[1]["stats"]["samples"]["total"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stats_worker, args=(r, 2, port, words, 5 * 64, q)) for r in range(2)]
    for p in procs:
        p.start()
    pixels, samples, bounces = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    fs = full["stats"]
    assert pixels == fs["pixels"]
    for k in ("total", "min", "max"):
        assert samples[k] == fs["samples"][k] and bounces[k] == fs["bounces"][k], k
    assert samples["avg"] == fs["samples"]["total"] / fs["pixels"]


def test_merge_stats_words_skips_empty_ranks_and_ors_errors():
    import torch
    from raytracer_amd.distributed import merge_stats_words, stats_from_words
    w = torch.tensor([[10, 40, 4, 4, 90, 1, 16, 0], [0, 0, -1, 0, 0, -1, 0, 0], [6, 24, 4, 4, 30, 0, 9, 0]])
    st = stats_from_words(merge_stats_words(w).tolist())
    assert (st.pixels, st.samples["total"], st.samples["min"], st.samples["max"]) == (16, 64, 4, 4)
    assert (st.bounces["total"], st.bounces["min"], st.bounces["max"]) == (120, 0, 16)
    empty = stats_from_words(merge_stats_words(w[1:2]).tolist())
    assert empty.samples["min"] == float("inf") and empty.bounces["min"] == float("inf")
    w[2, 7] = 2
    with pytest.raises(RuntimeError, match="emission stack"):
        stats_from_words(merge_stats_words(w).tolist())


def test_render_frame_orders_the_render_stream_after_the_gather_on_every_rank(monkeypatch):
    """on ranks above 0 the gather still reads `slab` on torch's current stream
    when render_frame returns; the caller's render stream must be made to wait for it (so a
    next render into a reused slab cannot overwrite it), as on rank 0. The device calls are
    stood in for; what is checked is the order of the stream hand-offs."""
    sys.path.insert(0, str(ROOT / "mcp-raytracer_amd"))
    from raytracer_amd import distributed as D

    calls = []

    class Cam:
        image_width, image_height = 16, 16

        def render_device(self, **kw):
            calls.append(("render", kw["stream"]))

        def stats_words(self, ptr, stream):
            calls.append(("stats", stream))

    class Slab:
        def numel(self):
            return 10 ** 6

        def data_ptr(self):
            return 0

    class Frame:
        device = "cuda:0"

    monkeypatch.setattr(D, "_wait", lambda s, d: calls.append(("wait", s)))
    monkeypatch.setattr(D, "_wait_for_current", lambda s, d: calls.append(("wait_for_current", s)))
    monkeypatch.setattr(D, "gather_slabs", lambda slab, world, out=None: calls.append(("gather",)) or None)
    assert D.render_frame(Cam(), Frame(), rank=1, world=2, stream=1234, slab=Slab()) is None
    names = [c[0] for c in calls]
    assert names == ["render", "stats", "wait", "gather", "wait_for_current"]
    assert calls[-1] == ("wait_for_current", 1234)


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 6, 7, 8, 16])
@pytest.mark.parametrize("W,H,region", [(800, 800, None), (37, 21, None), (64, 64, (3, 2, 59, 61)),
                                         (1920, 1080, (-5, 100, 700, 2000)), (8, 9, (0, 0, 8, 9)),
                                         (20, 20, (30, 0, 5, 5))])
def test_multi_plan_matches_the_tile_split(rt, n, W, H, region):
    """rt_multi_plan_region (the C ABI's single-process multi-GPU split, rt_camera_render_multi)
    against the Python restatement bench.py's one-process-per-GPU path uses: the same slab sizes,
    stats-word offset and per-device tile counts, and every region tile lands in exactly one slab
    slot that rt_tiles_unpack maps back to it (tile t -> entry t % n, slot t // n)."""
    from raytracer_amd import _lib
    from raytracer_amd import distributed as rtd
    region = region or (0, 0, W, H)
    p = _lib.multi_plan(region, W, H, n)
    reg = rtd.clamp_region(region, W, H)
    assert p["region"] == reg
    tiles = rtd.tile_count(reg)
    assert p["tiles"] == tiles and p["n_devices"] == n
    assert p["slab_tiles"] == rtd.slab_tiles(reg, n)
    assert p["slab_bytes_rgb"] == rtd.slab_pixels(reg, n) * 3
    assert p["slab_bytes_radiance"] == p["slab_tiles"] * 64 * 3 * 4
    assert p["stats_offset"] == p["slab_tiles"] * 64 * 3
    assert p["stats_offset"] + rtd.STATS_BYTES <= p["slab_bytes_rgb"]
    assert p["group_tiles"] == [len(rtd.owned_tiles(reg, g, n)) for g in range(n)]
    assert sum(p["group_tiles"]) == tiles and max(p["group_tiles"] + [0]) <= p["slab_tiles"]
    seen = set()
    for g in range(n):
        for k, t in enumerate(rtd.owned_tiles(reg, g, n)):
            assert t == g + k * n and k < p["slab_tiles"]  # frame.hip: region tile r + k * groups
            seen.add(t)
    assert seen == set(range(tiles))


def test_multi_plan_rejects_bad_device_counts(rt):
    from raytracer_amd import _lib
    for n in (0, -1, _lib.MAX_DEVICES + 1):
        with pytest.raises(_lib.RtError):
            _lib.multi_plan((0, 0, 8, 8), 8, 8, n)


def test_multi_stats_merge_matches_renderstats_merge(rt):
    """The merge rt_camera_render_multi applies to the devices' stats words (merge_stats_words,
    rt_api.cpp) is RenderStats.merge (renderStats.ts:42-64): restated here over random words and
    compared with the Python merge bench.py's per-rank path runs (distributed.merge_stats_words)."""
    import torch
    from raytracer_amd import distributed as rtd
    g = np.random.default_rng(7)
    for n in (1, 2, 5, 8):
        w = g.integers(0, 1 << 40, size=(n, 8), dtype=np.int64)
        w[:, 7] = 0
        w[g.random(n) < 0.3, 2] = -1  # a device without samples: minima ~0
        w[g.random(n) < 0.3, 5] = -1
        m = rtd.merge_stats_words(torch.from_numpy(w)).numpy()
        u = w.astype(np.uint64)
        assert m[0] == w[:, 0].sum() and m[1] == w[:, 1].sum() and m[4] == w[:, 4].sum()
        assert np.uint64(m[2]) == u[:, 2].min() and np.uint64(m[5]) == u[:, 5].min()
        assert m[3] == w[:, 3].max() and m[6] == w[:, 6].max()


def test_render_multi_without_a_device_fails_loudly(rt):
    """No GPU here: the multi-GPU entry returns an error (never a CPU fallback)."""
    if rt.device_count() > 0:
        pytest.skip("a device is visible")
    from raytracer_amd import _lib
    cam = rt.create_camera_from_scene_data(rt.generate_scene_data({"type": "cornell"}), {"width": 16, "samples": 1})
    buf = np.zeros((16, 16, 3), np.uint8)
    with pytest.raises(_lib.RtError):
        cam.render_multi(buf, [0, 1])
