"""bench.py host logic on the CPU: the algorithmic-bytes accounting
and the CPU baseline leg (oracle, one thread + all cores) on BASELINE config 1's
scene (spheres, count 10, 200x200, spp 4, depth 4 - the reference's own CPU case)."""
import pytest


def test_algorithmic_bytes_formula():
    import bench

    c = {"node": 1, "sphere": 2, "quad": 3, "plane": 4, "material": 5, "light_quad": 6, "light_sphere": 7}
    want = 32 * 1 + 16 * 2 + 64 * 3 + 64 * 4 + 32 * 5 + 64 * 6 + 16 * 7 + 12 * 10
    assert bench.algorithmic_bytes(c, 10) == pytest.approx(want)


def test_cpu_baseline_contract(rt):
    import bench

    sd = rt.generate_scene_data({"type": "spheres"})
    ropts = {"width": 40, "aspect": 1, "samples": 4, "depth": 4, "aTolerance": 0}
    line = bench.cpu_baseline(sd, ropts, 40, 40, 4, target_s=0.2)
    assert line["unit"] == "Msamples/s" and line["kind"] == "port" and line["cores"] == 1
    assert line["value"] > 0 and "single thread" in line["sample"]
    mc = line.get("multi_core")
    if mc is not None:  # hosts with more than one usable core
        assert mc["cores"] > 1 and mc["value"] > 0 and mc["unit"] == "Msamples/s"
        assert isinstance(mc["cpu"], str) and mc["cpu"]


def test_parity_check_accepts_the_oracle_frame_and_flags_one_pixel(rt, oracle):
    """bench.py's driver-observable parity leg on the CPU: fed the oracle's own
    frame it reports 0 / 0 differing pixels; one changed radiance value or u8
    byte on a checked row fails it; a timed frame that differs from the re-render
    fails it too."""
    from types import SimpleNamespace

    import bench
    from raytracer_amd.camera import RenderStats

    sd = rt.generate_scene_data({"type": "spheres"})
    ro = {"width": 40, "aspect": 1, "samples": 4, "depth": 4, "aTolerance": 0, "seed": 0x5EED}
    orc = oracle.render(sd, ro)
    fs = orc["stats"]
    st = RenderStats(pixels=fs["pixels"], samples=dict(fs["samples"]), bounces=dict(fs["bounces"]))
    args = SimpleNamespace(seed=0x5EED, spp=4, precision="ref")
    rgb, rad = orc["rgb"].copy(), orc["radiance"].copy()
    p = bench.parity_check(sd, {**ro, "precision": "ref", "traversal": "auto"}, args, rgb, rgb, rad, st)
    assert p["ok"] and p["pixels_differing_rgb"] == 0 and p["pixels_differing_radiance"] == 0
    assert p["pixels_checked"] == 40 * len(p["rows"]) and len(p["rows"]) >= 4
    j = p["rows"][1]
    bad = rad.copy()
    bad[j, 7, 1] = bad[j, 7, 1] * 1.0000001 + 1e-7
    q = bench.parity_check(sd, ro, args, rgb, rgb, bad, st)
    assert not q["ok"] and q["pixels_differing_radiance"] == 1 and q["rows"] == p["rows"]
    other = rgb.copy()
    other[(j + 1) % 40 if (j + 1) % 40 not in p["rows"] else 0, 0, 0] ^= 1
    r = bench.parity_check(sd, ro, args, other, rgb, rad, st)
    assert not r["ok"] and not r["timed_frame_equals_rerender"]


def test_bench_rejects_bad_repeat_counts():
    """--repeats 0 used to fail with IndexError after the whole warmup."""
    import bench
    for bad in (["--repeats", "0"], ["--steps", "0"], ["--warmup", "-1"], ["--gpus", "0"]):
        with pytest.raises(SystemExit):
            bench.parse_args(bad)
    a = bench.parse_args(["--single-process", "--gpus", "2", "--devices", "0,0"])
    assert a.single_process and a.devices == "0,0"
