#!/usr/bin/env python3
"""Benchmark: Msamples/s of the path-tracing hot path on the BASELINE.json
headline config (Cornell 800x800, spp=256, depth=16), 1..N GPUs.

One step = one full-image render (every pixel x spp paths) with the scene and
camera already resident in HBM, plus - for N > 1 - the RCCL gather of every
rank's tile-packed slab to rank 0 and its unpack into the frame. Rank 0 prints
one JSON line.

`python bench.py --gpus N` with N > 1 starts torch.distributed.run (one process
per GPU) as a child process before touching the GPU and forwards rank 0's line
and the exit code; under torch.distributed.run, WORLD_SIZE must equal --gpus.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "mcp-raytracer_amd"))

HEADLINE_METRIC = "Msamples/sec (w×h×spp/s) Cornell 800×800 spp=256 @1/2/4/8 GPU"  # BASELINE.json
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
SIMDS = 1024               # 256 CUs x 4 SIMD-32
CLOCK_GHZ = 2.4            # max engine clock (MI355X_MICROARCH.md)
# VALU issue peak: a SIMD-32 issues one wave64 VALU instruction per 2 cycles
# (MI355X_MICROARCH.md, wave scheduling), so 1024 x 2.4 GHz / 2 wave-instructions/s
VALU_PEAK_GINST = SIMDS * CLOCK_GHZ / 2.0

SCENES = {
    "cornell": ({"type": "cornell"}, {}, "Cornell"),
    "spheres": ({"type": "spheres", "options": {"count": 500, "seed": 42}}, {"aspect": 1}, "spheres-500"),
    "spheres10": ({"type": "spheres", "options": {"seed": 42}}, {"aspect": 1}, "spheres-10"),
    "rain": ({"type": "rain", "options": {"seed": 42}}, {}, "rain-50"),
    "default": ({"type": "default"}, {}, "default"),
    # BASELINE config 5: 100k requested, ~76.6k placed by the reference's rule
    "spheres100k": ({"type": "spheres", "options": {"count": 100000, "seed": 42}}, {"aspect": 1}, "spheres-100k"),
}


KERNEL_DESC = {
    "pool": "stage-compacted pool (per-wave LDS path slots, trace/diffuse queues, in-order accumulate)",
    "chunked": "chunked (lane work pool, in-order accumulate)",
}


def log(msg: str) -> None:
    """Progress on stderr (long runs must keep writing)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def metric_for(scene: str, W: int, H: int, spp: int, depth: int, adaptive: bool = False) -> str:
    if adaptive:
        return (f"Msamples/sec (traced samples/s, adaptive aTolerance=0.05 aBatch=10) {SCENES[scene][2]} "
                f"{W}×{H} spp≤{spp} depth={depth}")
    if (scene, W, H, spp, depth) == ("cornell", 800, 800, 256, 16):
        return HEADLINE_METRIC
    return f"Msamples/sec (w×h×spp/s) {SCENES[scene][2]} {W}×{H} spp={spp} depth={depth}"


def algorithmic_bytes(c: dict, pixels: int) -> float:
    """32 B/node + 16 B/sphere test + 64 B/quad or plane test +
    32 B/material fetch + per diffuse bounce per light (64 quad | 16 sphere)
    + 12 B/pixel accumulator write."""
    return (32.0 * c["node"] + 16.0 * c["sphere"] + 64.0 * c["quad"] + 64.0 * c["plane"]
            + 32.0 * c["material"] + 64.0 * c["light_quad"] + 16.0 * c["light_sphere"] + 12.0 * pixels)


def cpu_baseline(scene_data, ropts, width, height, spp, target_s=15.0):
    """The CPU restatement (oracle, ref precision, 1 thread) on a bounded row
    subsample of the same workload. The oracle restates the reference's object
    model (virtual Hittable.hit / Material.scatter, a recursive rayColor, a
    MixturePDF allocated per diffuse bounce, as src/camera.ts:263-315 does): the
    stand-in for the single-threaded TypeScript path, which cannot run here
    (SURVEY.md §8c). Beside it: the same restatement over the host cores
    (`multi_core`) and in fp32 scalars (`fp32`, BASELINE.md §4's row)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import pyoracle

    pyoracle.build()
    # one short row segment sizes the sample: (cost per pixel) -> rows that fit target_s
    seg = min(width, 64)
    t0 = time.perf_counter()
    pyoracle.render(scene_data, ropts, region=((width - seg) // 2, height // 2, seg, 1), threads=1)
    t_px = max(time.perf_counter() - t0, 1e-4) / seg
    rows = max(1, min(height, int(target_s / (t_px * width))))
    step = max(1, height // rows)
    region = None
    if t_px * width > target_s:  # one full row is already too long: a centred row segment
        n = max(8, int(target_s / t_px))
        region, step = ((width - n) // 2, height // 2, n, 1), 1
    t0 = time.perf_counter()
    out = pyoracle.render(scene_data, ropts, row_step=step, threads=1, region=region)
    dt = time.perf_counter() - t0
    samples = out["stats"]["samples"]["total"]
    what = (f"rows j%{step}==0 of the {width}x{height} image" if region is None
            else f"{region[2]} px of row {region[1]}")
    line = {"value": samples / dt / 1e6, "unit": "Msamples/s", "cores": 1, "kind": "port",
            "sample": f"{what} at spp={spp} ({int(out['stats']['pixels'])} px, {int(samples)} samples, "
                      f"{dt:.1f} s), oracle/oracle.cpp ref precision (the reference's object model: virtual "
                      f"hit/scatter, per-bounce MixturePDF allocation), single thread"}
    # the same restatement with fp32 scalars, single thread, about half the work
    step32 = step * 2
    t0 = time.perf_counter()
    out = pyoracle.render(scene_data, ropts, row_step=step32, threads=1, region=region, precision="fp32")
    dt32 = time.perf_counter() - t0
    s32 = out["stats"]["samples"]["total"]
    line["fp32"] = {"value": s32 / dt32 / 1e6, "unit": "Msamples/s", "cores": 1,
                    "sample": f"rows j%{step32}==0 ({int(s32)} samples, {dt32:.1f} s), oracle/oracle.cpp fp32 "
                              f"scalars, single thread" if region is None else
                              f"{region[2]} px of row {region[1]} ({int(s32)} samples, {dt32:.1f} s), fp32 scalars"}
    # the same restatement over all of this process's host cores
    # (threads over rows, the analogue of the reference's -p workers), ~target_s/2 of work.
    # The GPU box grants a 16-CPU share whatever nproc says.
    cores = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
    if cores > 1 and region is None:
        step_mt = max(1, step * 2 // cores)
        t0 = time.perf_counter()
        out = pyoracle.render(scene_data, ropts, row_step=step_mt, threads=cores)
        dt = time.perf_counter() - t0
        s_mt = out["stats"]["samples"]["total"]
        line["multi_core"] = {"value": s_mt / dt / 1e6, "unit": "Msamples/s", "cores": cores,
                              "cpu": _cpu_model(),
                              "sample": f"rows j%{step_mt}==0 ({int(s_mt)} samples, {dt:.1f} s), "
                                        f"{cores} threads over rows"}
    return line


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_children(args, argv) -> int:
    """--gpus N > 1 without a torch.distributed.run environment: run N ranks as a
    child process (never exec from this process) and forward rank 0's output."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(Path(__file__).resolve()), *argv]
    log("launching " + " ".join(cmd[2:6]) + " ...")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def parse_args(argv):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--repeats", type=int, default=3,
                    help="timed repeats of --steps steps; the median repeat is reported (SURVEY.md §8d)")
    ap.add_argument("--scene", default="cornell", choices=sorted(SCENES))
    ap.add_argument("--width", type=int, default=800)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--depth", type=int, default=16)
    ap.add_argument("--precision", default="ref", choices=["ref", "fp32"])
    ap.add_argument("--seed", type=int, default=0x5EED)
    ap.add_argument("--traversal", default="auto", choices=["auto", "brute", "fast", "reference"],
                    help="closest-hit strategy (all bit-identical; auto = brute force up to 16 primitives)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-count", action="store_true", help="skip the work-counting launch (no work_rate)")
    ap.add_argument("--no-parity", action="store_true", help="skip the oracle rows check of the timed frame")
    ap.add_argument("--adaptive", action="store_true",
                    help="adaptive sampling with the reference's defaults (aTolerance 0.05, aBatch 10)")
    ap.add_argument("--count-sub", type=int, default=0,
                    help="tile subsample of the work-counting launch (0 = auto: 16 above 1000 objects)")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N > 1 (nccl = RCCL)")
    ap.add_argument("--check", action="store_true",
                    help="rank 0 compares the assembled frame with a single-launch render of the whole image")
    ap.add_argument("--stub", action="store_true",
                    help="CPU rehearsal of the launcher and the gather (gloo, no GPU, no render: tests only)")
    ap.add_argument("--single-process", action="store_true",
                    help="one process drives all N GPUs through the C ABI's rt_camera_render_multi (the call the "
                         "TypeScript host makes through the N-API addon): host frame out, RCCL gather inside")
    ap.add_argument("--devices", default="",
                    help="--single-process: comma-separated device ordinals (default 0..N-1; a repeated ordinal "
                         "rehearses the N-way split on fewer GPUs)")
    a = ap.parse_args(argv)
    if a.repeats < 1 or a.steps < 1 or a.warmup < 0 or a.gpus < 1:
        ap.error("--repeats and --steps must be >= 1, --warmup >= 0, --gpus >= 1")
    return a


def _load_profile(name: str, key: str):
    f = ROOT / "profiles" / name
    if not f.exists():
        return None
    try:
        return json.loads(f.read_text()).get(key)
    except Exception:
        return None


def roofline(cfg_key: str, build: str, samples: int, kernel_ms: float, counters, pixels: int):
    """The dominant kernel against the bound it sits on: VALU issue.

    achieved = VALU wave64 instructions per sample (rocprofv3 SQ_INSTS_VALU of
    the same configuration and build, profiles/pmc_valu.json) x this launch's
    samples / the launch's kernel time measured here with HIP events on the
    launch stream; peak = 1024 SIMDs x 2.4 GHz / 2 cycles. `lane_util` (active
    lanes per issued instruction, SQ_THREAD_CYCLES_VALU / 64 SQ_ACTIVE_INST_VALU)
    times frac is the useful lane-issue fraction. `hbm` = the measured HBM bytes
    of the same kernel (FETCH_SIZE x 2 + WRITE_SIZE, separate --pmc passes,
    profiles/pmc_traffic.json) over the same time. `work_rate` = SURVEY.md §8d's
    algorithmic bytes (L1/LDS-resident scene reads, not HBM) over the same time."""
    k_s = kernel_ms / 1e3
    v = _load_profile("pmc_valu.json", cfg_key)
    t = _load_profile("pmc_traffic.json", cfg_key)
    out = {"bound": "valu", "unit": "Ginst/s", "peak": VALU_PEAK_GINST, "kernel_ms": round(kernel_ms, 4)}
    if v:
        ips = v["valu_insts_per_sample"] / 64.0  # wave instructions per sample
        ach = ips * samples / k_s / 1e9
        # issue-weighted: an f64 add / mul / fma issues at half the f32 rate on gfx950
        # (78.6 vs 157.3 TFLOP/s) and a transcendental at a quarter, so those instructions hold
        # the SIMD 2x / 4x as long as `frac` counts them (mix: their shares of SQ_INSTS_VALU)
        mix = v.get("mix", {})
        w = (1.0 + sum(mix.get(k, 0.0) for k in ("add_f64", "mul_f64", "fma_f64"))
             + 3.0 * (mix.get("trans_f32", 0.0) + mix.get("trans_f64", 0.0)))
        out.update({"achieved": round(ach, 2), "frac": round(ach / VALU_PEAK_GINST, 4),
                    "frac_issue_weighted": round(ach * w / VALU_PEAK_GINST, 4),
                    "issue_weights": {"f64_add_mul_fma": 2, "transcendental": 4, "factor": round(w, 4)},
                    "lane_util": v["lane_util"], "useful_lane_frac": round(ach / VALU_PEAK_GINST * v["lane_util"], 4),
                    "valu_wave_insts_per_sample": round(ips, 2),
                    "pmc_kernel": v["kernel"], "pmc_build": v.get("build_id"), "pmc_stale": v.get("build_id") != build,
                    "pmc_source": "profiles/pmc_valu.json"})
        assert out["frac"] <= 1.0, out
    else:
        out.update({"achieved": None, "frac": None, "pmc_source": None})
    traffic = t.get("hbm_bytes_per_launch") if t else None
    out["traffic"] = traffic
    if traffic:
        gbs = traffic / k_s / 1e9
        out["hbm"] = {"achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "frac": round(gbs / HBM_PEAK_GBS, 4), "pmc_build": t.get("build_id"),
                      "pmc_source": "profiles/pmc_traffic.json"}
    if counters:
        ab = algorithmic_bytes(counters, pixels)
        out["work_rate"] = {"algorithmic_bytes_per_launch": ab, "GBps": round(ab / k_s / 1e9, 1),
                            "note": "SURVEY.md §8d byte model of the reference algorithm (scene reads are "
                                    "LDS/L1-resident): a work rate, not HBM traffic",
                            "per_sample": {k: round(val / max(counters["samples"], 1), 3)
                                           for k, val in counters.items()}}
    return out


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if args.single_process:
        if env_world not in (None, "1"):
            print("bench.py: --single-process runs without torch.distributed.run", file=sys.stderr)
            return 2
        return single_process_main(args)
    if env_world is None and args.gpus > 1:
        return launch_children(args, argv)
    world_env = int(env_world or "1")
    if world_env != args.gpus:
        print(f"bench.py: WORLD_SIZE={world_env} but --gpus {args.gpus}", file=sys.stderr)
        return 2
    if args.stub:
        return stub_main(args)

    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # one GPU per rank; more ranks than devices (a CPU-backend rehearsal on one GPU) share them
    dev_index = local_rank % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    world = 1
    if world_env > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.backend)
        world = dist.get_world_size()  # the ranks RCCL actually connected
    from raytracer_amd import _build

    if rank == 0:
        _build.build_native()
    if world > 1:
        dist.barrier()
    import raytracer_amd as rt
    from raytracer_amd import distributed as rtd

    cfg, extra, _ = SCENES[args.scene]
    scene_data = rt.generate_scene_data(cfg)
    # --adaptive: the reference's default RenderOptions (aTolerance 0.05, aBatch 10;
    # src/camera.ts:77-78), which every reference caller keeps on
    adapt = {"aTolerance": 0.05, "aBatch": 10} if args.adaptive else {"aTolerance": 0}
    ropts = {"width": args.width, "samples": args.spp, "depth": args.depth, **adapt,
             "seed": args.seed, "precision": args.precision, "traversal": args.traversal, **extra}
    cam = rt.create_camera_from_scene_data(scene_data, ropts)
    W, H = cam.image_width, cam.image_height
    frame = torch.zeros((H, W, 3), dtype=torch.uint8, device=dev)
    # t_render ends with the frame on host rank 0 - every timed step
    # copies rank 0's u8 frame into this pinned buffer
    host_frame = torch.zeros((H, W, 3), dtype=torch.uint8, pin_memory=True) if rank == 0 else None
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    region = (0, 0, W, H)
    n_slab = rtd.slab_pixels(region, world)  # this rank's tiles + the spare tile carrying its stats words
    slab = torch.zeros((n_slab, 3), dtype=torch.uint8, device=dev) if world > 1 else None
    gathered = torch.zeros((world, n_slab, 3), dtype=torch.uint8, device=dev) if world > 1 and rank == 0 else None
    log(f"rank {rank}/{world}: {args.scene} {W}x{H} spp={args.spp} depth={args.depth} build {rt.build_id()}")

    # Algorithmic work of this rank's launch: the node / primitive /
    # material / light-PDF work the REFERENCE algorithm does on this workload,
    # counted by one instrumented, untimed launch with the reference-order
    # traversal (its counts equal the oracle's: test_work_counters_match_oracle),
    # on min(spp, 64) samples and, for large scenes, a 1/count_sub tile subsample.
    counters = None
    sub = args.count_sub or (16 if cam.info["n_objects"] > 1000 else 1)
    if not args.no_count:
        spp_c = min(args.spp, 64)
        cam_c = rt.create_camera_from_scene_data(scene_data, {**ropts, "samples": spp_c})
        st_c, counters = cam_c.render_device(rgb_ptr=frame.data_ptr(), tile_group=rank, tile_groups=world * sub,
                                             stream=sptr, synchronize=True, count_work=True,
                                             traversal="reference")
        cam_c.close()
        log(f"work counters: {int(st_c.samples['total'])} samples counted")

    # Rank 0's frame goes to pinned host memory on a copy stream, double-buffered: frame k's D2H
    # copy overlaps frame k+1's render (which writes the other device frame), and frame k+2 waits
    # for frame k's copy before it reuses its buffer. Every timed frame still reaches the host
    # inside the timed region (the closing synchronize waits for the copy stream too).
    frames = [frame, torch.zeros_like(frame)] if rank == 0 else [frame, frame]
    host_frames = [host_frame, torch.zeros_like(host_frame, pin_memory=True)] if rank == 0 else None
    copy_stream = torch.cuda.Stream(dev) if rank == 0 else None
    rendered = [torch.cuda.Event(), torch.cuda.Event()]
    copied = [torch.cuda.Event(), torch.cuda.Event()]  # (waiting on a never-recorded event is a no-op)
    nstep = [0]

    def step():
        b = nstep[0] % 2
        nstep[0] += 1
        if rank == 0:
            stream.wait_event(copied[b])  # frame k-2's copy has read this buffer
        fr = frames[b]
        if world == 1:
            cam.render_device(rgb_ptr=fr.data_ptr(), stream=sptr)
        else:
            rtd.render_frame(cam, fr, rank, world, stream=sptr, slab=slab, gathered=gathered)
        if rank == 0:
            rendered[b].record(stream)
            copy_stream.wait_event(rendered[b])
            with torch.cuda.stream(copy_stream):
                host_frames[b].copy_(fr, non_blocking=True)  # D2H inside the timed step
            copied[b].record(copy_stream)

    # this rank's share (untimed): pixels and samples per launch
    st, _ = cam.render_device(rgb_ptr=frame.data_ptr(), tile_group=rank, tile_groups=world, stream=sptr,
                              synchronize=True)
    my_pixels, my_samples = int(st.pixels), int(st.samples["total"])
    if counters:
        scale = my_samples / max(counters["samples"], 1)
        counters = {k: v * scale for k, v in counters.items()}
    for i in range(args.warmup):
        step()
        torch.cuda.synchronize()
        log(f"warmup {i + 1}/{args.warmup}")
    # three repeats, the median reported. Each repeat times exactly `steps`
    # steps between a barrier + synchronize on both sides; the max over ranks is taken per repeat.
    reps = []
    for r in range(args.repeats):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            step()
            if args.steps <= 5 or (i + 1) % 10 == 0:  # no sync here: keep launches queued
                log(f"repeat {r + 1}/{args.repeats}: step {i + 1}/{args.steps} queued")
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        reps.append(time.perf_counter() - t0)

    # Kernel time of the dominant kernel, from HIP events the library records on
    # the launch stream (per pass, path kernel and accumulate separately), over
    # untimed renders of this rank's share after the timed region.
    kt = []
    for _ in range(max(3, min(args.steps, 10))):
        cam.render_device(rgb_ptr=(slab if world > 1 else frame).data_ptr(), tile_group=rank, tile_groups=world,
                          stream=sptr, packed=world > 1)
        kt.append(cam.kernel_times())
    passes = cam.pass_count()
    a_rounds, a_rendered = cam.adaptive_info()
    kernel_ms = sum(a for a, _ in kt) / len(kt)
    accum_ms = sum(b for _, b in kt) / len(kt)
    kind = cam.last_kernel()  # the path kernel the library launched (rt_camera_last_kernel)
    kernel_name = {"pool": "pt_pool_kernel", "chunked": "pt_chunk_kernel"}.get(kind, "pt_render_kernel")

    t = torch.tensor([*reps, kernel_ms], dtype=torch.float64, device=dev if args.backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    reps = [float(x) for x in t[:len(reps)]]
    elapsed = sorted(reps)[len(reps) // 2]  # the median repeat (max over ranks)

    # Untimed: the same frame again with its fp32 radiance (assembled over the ranks
    # like the timed frames) and the merged RenderStats, for the checks below.
    radiance = torch.zeros((H, W, 3), dtype=torch.float32, device=dev)
    timed_rgb = host_frames[(nstep[0] - 1) % 2].numpy().copy() if rank == 0 else None
    res = rtd.render_frame(cam, frame, rank, world, stream=sptr, radiance=radiance, stats=True)
    torch.cuda.synchronize()
    frame_check = None
    if args.check:
        if rank == 0:
            single = torch.zeros_like(frame)
            st1, _ = cam.render_device(rgb_ptr=single.data_ptr(), stream=sptr, synchronize=True)
            frame_check = bool(torch.equal(single, frame)) and _stats_equal(res[1], st1)
            log(f"frame check (assembled frame and merged stats == single launch): {frame_check}")
    parity = None
    if rank == 0 and not args.no_parity:
        parity = parity_check(scene_data, ropts, args, timed_rgb, frame.cpu().numpy(), radiance.cpu().numpy(),
                              res[1])
    if world > 1:
        dist.barrier()

    if rank == 0:
        # samples traced per frame (merged over the ranks): W*H*spp at fixed spp; fewer
        # with adaptive sampling, where pixels stop once converged
        samples_per_step = int(res[1].samples["total"])
        value = samples_per_step * args.steps / elapsed / 1e6
        key = f"{args.scene}_{W}x{H}_spp{args.spp}_d{args.depth}_{args.precision}_n{world}" + \
            ("_adaptive" if args.adaptive else "")
        rl = roofline(key, rt.build_id(), my_samples, kernel_ms, counters, my_pixels)
        rl.update({"kernel": kernel_name, "accum_kernel_ms": round(accum_ms, 4), "passes": passes,
                   "count_subsample": sub})
        if accum_ms > 0 and not args.adaptive:
            # the in-order accumulate pass (pt_accum_kernel) is the HBM-bound kernel of the frame: it
            # streams every sample's record (12 B {r, g, b} at fixed spp in colour mode, 16 B with
            # the bounce word) once and writes each pixel's u8 RGB (3 B); algorithmic bytes / its time
            rec_b = 16 if cam.info["mode"] == 1 else 12  # MODE_BOUNCES keeps the bounce word
            ab = my_samples * rec_b + my_pixels * 3
            gbs = ab / (accum_ms / 1e3) / 1e9
            rl["accumulate"] = {"kernel": "pt_accum_kernel", "bound": "hbm", "achieved": round(gbs, 1),
                                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                                "algorithmic_bytes_per_launch": ab, "record_bytes_per_sample": rec_b}
        if args.adaptive:
            rl["adaptive_rounds"] = {"rounds": a_rounds, "samples_rendered": a_rendered,
                                     "samples_kept": int(my_samples),
                                     "speculation": round(a_rendered / max(my_samples, 1) - 1.0, 4)}
        cpu = None
        if world == 1 and not args.no_cpu:
            log("cpu baseline")
            cpu = cpu_baseline(scene_data, {k: v for k, v in ropts.items() if k not in ("precision", "traversal")},
                               W, H, args.spp)
        line = {
            "metric": metric_for(args.scene, W, H, args.spp, args.depth, args.adaptive), "value": round(value, 3),
            "unit": "Msamples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "repeats": {"n": len(reps), "reported": "median",
                        "ms_per_step": [round(x / args.steps * 1e3, 3) for x in reps]},
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "f64" if args.precision == "ref" else "f32",
            "data": "synthetic: reference scene generator output (deterministic), path RNG seed "
                    f"{args.seed:#x}; no datasets",
            "config": {"workload": f"{args.scene} {W}x{H} spp={args.spp} depth={args.depth}",
                       "scene": args.scene, "width": W, "height": H, "spp": args.spp, "depth": args.depth,
                       "precision": args.precision, "adaptive": adapt if args.adaptive else False,
                       "samples_per_frame": samples_per_step,
                       "traversal": ["fast", "reference", "brute"][cam.info["traversal"]],
                       "kernel": KERNEL_DESC.get(kind, "sequential (wave per 8x8 tile)"),
                       "parallelism": f"8x8-tile interleave x{world}" +
                                      (" + RCCL gather of tile-packed slabs to rank 0" if world > 1 else "")},
            "build_id": rt.build_id(),
            **({"frame_check": frame_check} if args.check else {}),
            "host_copy": "each timed step copies rank 0's u8 frame into pinned host memory (copy stream, "
                         "double-buffered: frame k's copy overlaps frame k+1's render; all inside the timed region)",
            "parity": parity,
            "roofline": rl,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    rc = 0
    if rank == 0 and parity is not None and not parity["ok"]:
        log("PARITY FAILURE: the timed frame differs from the oracle")
        rc = 3
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return rc


def single_process_main(args) -> int:
    """--single-process: one process renders each frame over N GPUs with ONE C-ABI call,
    rt_camera_render_multi (tile groups per device on their own streams, RCCL gather of the
    tile-packed slabs on devices[0], unpack, merged stats, frame copied into the caller's host
    buffer) - what the TypeScript host's generateImageBuffer does through the N-API addon's
    renderRegionMulti (src/raytracer.ts:60-90 replaced by one call). A step = one frame,
    host buffer included, exactly as the per-rank path's step ends with the host copy."""
    import numpy as np
    import torch

    from raytracer_amd import _build

    _build.build_native()
    import raytracer_amd as rt

    n_vis = rt.device_count()
    devices = [int(d) for d in args.devices.split(",")] if args.devices else list(range(args.gpus))
    if len(devices) != args.gpus:
        print(f"bench.py: --devices lists {len(devices)} ordinals for --gpus {args.gpus}", file=sys.stderr)
        return 2
    if max(devices) >= n_vis:
        print(f"bench.py: devices {devices} but {n_vis} visible", file=sys.stderr)
        return 2
    cfg, extra, _ = SCENES[args.scene]
    scene_data = rt.generate_scene_data(cfg)
    adapt = {"aTolerance": 0.05, "aBatch": 10} if args.adaptive else {"aTolerance": 0}
    ropts = {"width": args.width, "samples": args.spp, "depth": args.depth, **adapt,
             "seed": args.seed, "precision": args.precision, "traversal": args.traversal, **extra}
    cam = rt.create_camera_from_scene_data(scene_data, ropts)
    W, H = cam.image_width, cam.image_height
    region = (0, 0, W, H)
    host_frame = torch.zeros((H, W, 3), dtype=torch.uint8, pin_memory=True).numpy()
    log(f"single process: {args.scene} {W}x{H} spp={args.spp} depth={args.depth} on devices {devices} "
        f"build {rt.build_id()}")
    for i in range(args.warmup):
        cam.render_region_multi(host_frame, region, devices)
        log(f"warmup {i + 1}/{args.warmup}")
    reps = []
    for r in range(args.repeats):
        t0 = time.perf_counter()
        for i in range(args.steps):
            st = cam.render_region_multi(host_frame, region, devices)  # returns with the frame in host memory
            if args.steps <= 5 or (i + 1) % 10 == 0:
                log(f"repeat {r + 1}/{args.repeats}: step {i + 1}/{args.steps}")
        reps.append(time.perf_counter() - t0)
    elapsed = sorted(reps)[len(reps) // 2]
    info = cam.multi_info()
    timed_rgb = host_frame.copy()
    kernel_ms = max(info["path_ms"])
    rad = np.zeros((H, W, 3), np.float32)
    rgb = np.zeros((H, W, 3), np.uint8)
    res = cam.render_region_multi(rgb, region, devices, radiance=rad)
    parity = None if args.no_parity else parity_check(scene_data, ropts, args, timed_rgb, rgb, rad, res)
    samples_per_step = int(res.samples["total"])
    value = samples_per_step * args.steps / elapsed / 1e6
    n_dev = len(set(devices))
    key = f"{args.scene}_{W}x{H}_spp{args.spp}_d{args.depth}_{args.precision}_n1" + ("_adaptive" if args.adaptive else "")
    # one device: the dominant kernel against VALU issue as in the per-rank path; several: the
    # slowest device's path kernel (its share's counters are not collected separately)
    rl = (roofline(key, rt.build_id(), samples_per_step, kernel_ms, None, W * H) if len(devices) == 1 else
          {"bound": "valu", "kernel_ms": round(kernel_ms, 4), "frac": None,
           "note": "slowest device's path kernel; per-device times in `multi`"})
    line = {
        "metric": metric_for(args.scene, W, H, args.spp, args.depth, args.adaptive), "value": round(value, 3),
        "unit": "Msamples/s", "n_gpus": n_dev, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "repeats": {"n": len(reps), "reported": "median", "ms_per_step": [round(x / args.steps * 1e3, 3) for x in reps]},
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "dtype": "f64" if args.precision == "ref" else "f32",
        "data": f"synthetic: reference scene generator output (deterministic), path RNG seed {args.seed:#x}; no datasets",
        "config": {"workload": f"{args.scene} {W}x{H} spp={args.spp} depth={args.depth}", "scene": args.scene,
                   "width": W, "height": H, "spp": args.spp, "depth": args.depth, "precision": args.precision,
                   "adaptive": adapt if args.adaptive else False, "samples_per_frame": samples_per_step,
                   "parallelism": f"single process, rt_camera_render_multi over devices {devices}: 8x8-tile "
                                  f"interleave, {info['transport']} gather of tile-packed slabs on device "
                                  f"{devices[0]}, host frame out"},
        "build_id": rt.build_id(),
        "multi": {"transport": info["transport"], "devices": devices,
                  "path_ms": [round(x, 4) for x in info["path_ms"]],
                  "accum_ms": [round(x, 4) for x in info["accum_ms"]], "gather_ms": round(info["gather_ms"], 4),
                  "slab_tiles": info["slab_tiles"]},
        "host_copy": "each timed step is one rt_camera_render_multi call returning with the u8 frame in host memory",
        "parity": parity,
        "roofline": rl,
        "cpu_baseline": None,
    }
    print(json.dumps(line), flush=True)
    if parity is not None and not parity["ok"]:
        log("PARITY FAILURE: the timed frame differs from the oracle")
        return 3
    return 0


def _stats_equal(a, b) -> bool:
    return (a.pixels == b.pixels and all(a.samples[k] == b.samples[k] for k in ("total", "min", "max"))
            and all(a.bounces[k] == b.bounces[k] for k in ("total", "min", "max")))


def parity_check(scene_data, ropts, args, timed_rgb, rgb, rad, stats, row_budget_s=4.0):
    """Driver-observable parity (after the timed region, never inside it): rows of
    the frame chosen from the seed, re-rendered by the CPU oracle (same seed, same
    precision mode) and compared bit for bit - u8 of the LAST TIMED frame as it
    reached host memory, and the fp32 radiance of an untimed re-render whose u8
    must equal the timed frame. Rows are full rows when the oracle can render one
    in ~row_budget_s, else a seeded segment of each. ref precision: exact; fp32:
    SURVEY.md §8c's tolerance (>= 99 % of pixels within 1e-3 + 1e-3|c|).
    Reference loop: src/camera.ts:388-431."""
    import random
    from concurrent.futures import ThreadPoolExecutor

    import numpy as np

    sys.path.insert(0, str(ROOT / "oracle"))
    import pyoracle

    pyoracle.build()
    H, W = rgb.shape[:2]
    o_ro = {k: v for k, v in ropts.items() if k not in ("precision", "traversal")}
    rnd = random.Random(args.seed * 7919 + W * 31 + H)
    t_start = time.perf_counter()
    # pilot: oracle cost per pixel on 8 pixels of the middle row
    t0 = time.perf_counter()
    pyoracle.render(scene_data, o_ro, region=(W // 2 - 4 if W >= 8 else 0, H // 2, min(8, W), 1),
                    precision="ref")
    t_px = max(time.perf_counter() - t0, 1e-4) / min(8, W)
    cores = max(1, min(len(os.sched_getaffinity(0)), 16))
    n_rows = min(H, 8 if t_px * W * 8 <= cores * row_budget_s else 4)
    rows = sorted(rnd.sample(range(H), n_rows))
    seg = min(W, max(8, int(row_budget_s / t_px)))
    xs = [0 if seg == W else rnd.randrange(0, W - seg + 1) for _ in rows]

    def one(k):
        return pyoracle.render(scene_data, o_ro, region=(xs[k], rows[k], seg, 1), precision="ref")

    with ThreadPoolExecutor(max_workers=min(cores, n_rows)) as ex:
        outs = list(ex.map(one, range(n_rows)))
    n_rgb = n_rad = n_px = n_tol = 0
    for k, o in enumerate(outs):
        j, x0 = rows[k], xs[k]
        a_rgb, a_rad = timed_rgb[j, x0:x0 + seg], rad[j, x0:x0 + seg]
        b_rgb, b_rad = o["rgb"][j, x0:x0 + seg], o["radiance"][j, x0:x0 + seg]
        n_px += seg
        n_rgb += int((a_rgb != b_rgb).any(axis=-1).sum())
        same = (a_rad == b_rad) | (np.isnan(a_rad) & np.isnan(b_rad))
        n_rad += int((~same).any(axis=-1).sum())
        d = np.abs(a_rad.astype(np.float64) - b_rad)
        n_tol += int((d <= 1e-3 + 1e-3 * np.abs(b_rad)).all(axis=-1).sum())
    timed_eq = bool(np.array_equal(timed_rgb, rgb))
    full = stats.pixels == W * H and (stats.samples["total"] == W * H * args.spp if not ropts.get("aTolerance")
                                      else 0 < stats.samples["total"] <= W * H * args.spp)
    if args.precision == "ref":
        ok = n_rgb == 0 and n_rad == 0 and timed_eq and bool(full)
        rule = "bit-exact (u8 and fp32 radiance)"
    else:
        ok = n_tol >= 0.99 * n_px and timed_eq and bool(full)
        rule = "SURVEY.md §8c: >= 99 % of pixels within 1e-3 + 1e-3|c|"
    out = {"ok": ok, "rule": rule, "rows": rows, "x": xs if seg < W else 0, "width": seg,
           "pixels_checked": n_px, "pixels_differing_rgb": n_rgb, "pixels_differing_radiance": n_rad,
           "pixels_within_tolerance": n_tol, "timed_frame_equals_rerender": timed_eq,
           "stats": {"pixels": stats.pixels, "samples": stats.samples["total"], "bounces": stats.bounces["total"],
                     "bounces_max": stats.bounces["max"]},
           "oracle": f"oracle/oracle.cpp ref precision, {min(cores, n_rows)} threads",
           "seconds": round(time.perf_counter() - t_start, 2)}
    log(f"parity: {n_px} px on rows {rows}: rgb {n_rgb}, radiance {n_rad} differing; timed == rerender {timed_eq}")
    return out


def stub_main(args) -> int:
    """CPU rehearsal (tests): the same rank bookkeeping and slab gather over
    gloo, with a stand-in render that writes each owned pixel's own index into
    its slab; rank 0 checks the reassembled frame and prints a line like the
    real one. No GPU, no librt_amd.so."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from raytracer_amd import distributed as rtd

    rank = int(os.environ.get("RANK", "0"))
    world = 1
    if args.gpus > 1:
        dist.init_process_group("gloo")
        world = dist.get_world_size()
    W = H = args.width
    region = (0, 0, W, H)
    n_px = rtd.slab_tiles(region, world) * rtd.TILE_PIXELS
    tiles_x = -(-W // rtd.TILE)
    slab = np.zeros((n_px, 3), np.uint8)
    for k, g in enumerate(rtd.owned_tiles(region, rank, world)):
        ty, tx = divmod(g, tiles_x)
        for l in range(rtd.TILE_PIXELS):
            i, j = tx * rtd.TILE + l % rtd.TILE, ty * rtd.TILE + l // rtd.TILE
            if i < W and j < H:
                slab[k * rtd.TILE_PIXELS + l] = ((j * W + i) % 251, (j * W + i) // 251 % 251, rank)
    t0 = time.perf_counter()
    g = rtd.gather_slabs(torch.from_numpy(slab), world)
    elapsed = time.perf_counter() - t0
    if rank == 0:
        frame = np.zeros((H, W, 3), np.uint8)
        g = g.numpy()
        for r in range(world):
            for k, t in enumerate(rtd.owned_tiles(region, r, world)):
                ty, tx = divmod(t, tiles_x)
                for l in range(rtd.TILE_PIXELS):
                    i, j = tx * rtd.TILE + l % rtd.TILE, ty * rtd.TILE + l // rtd.TILE
                    if i < W and j < H:
                        frame[j, i] = g[r, k * rtd.TILE_PIXELS + l]
        idx = np.arange(W * H).reshape(H, W)
        ok = bool((frame[..., 0] == idx % 251).all() and (frame[..., 1] == idx // 251 % 251).all())
        owner = np.zeros((H, W), np.uint8)
        for r in range(world):
            owner[rtd.owner_mask(W, H, region, r, world)] = r
        ok = ok and bool((frame[..., 2] == owner).all())
        print(json.dumps({"metric": "stub", "value": 0.0, "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": round(elapsed * 1e3, 3), "stub_frame_ok": ok,
                          "slab_bytes_per_rank": int(slab.nbytes), "frame_bytes": W * H * 3}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
