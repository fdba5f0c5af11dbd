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
