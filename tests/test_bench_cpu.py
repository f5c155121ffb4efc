"""bench.py's measurement bookkeeping, on the CPU: the kernel-code digest that
ties a PMC profile to the launched kernel, the traffic attachment rule
(roofline.traffic only from a profile of the same variant and code), the
roofline figures and the GPU/CPU summary."""
import json
import os
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_code_digest_ignores_comments_only():
    src = "int a = 1; // one\n/* block\n comment */ float b = 2.0f;\n\n"
    same = "int a = 1; // another note\n/* x */ float b = 2.0f;\n"
    other = "int a = 2; // one\n/* block\n comment */ float b = 2.0f;\n"
    assert bench._code_only(src) == bench._code_only(same)
    assert bench._code_only(src) != bench._code_only(other)


def test_digest_per_traversal():
    b, v = bench.kernel_source_digest("brute"), bench.kernel_source_digest("bvh")
    assert len(b) == 64 and len(v) == 64 and b != v
    assert bench.kernel_source_digest("brute") == b  # deterministic


@pytest.fixture
def profile_dir(tmp_path, monkeypatch):
    os.makedirs(tmp_path / "profiles")
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "kernel_source_digest", lambda traversal="brute": f"digest-{traversal}")
    return tmp_path / "profiles"


def write_profile(d, config, variant, digest, hbm=1234560000):
    with open(d / f"pmc_config{config}.json", "w") as f:
        json.dump({"config": config, "kernel_variant": variant, "kernel_source_sha256": digest,
                   "hbm_bytes_per_launch": hbm}, f)


def test_traffic_attached_only_for_the_same_kernel(profile_dir):
    rf = bench.roofline(1e9, 0, 100.0)
    bench.attach_traffic(rf, "B", "smem/x", 100.0)
    assert rf["traffic"] is None and "no PMC profile" in rf["traffic_note"]

    write_profile(profile_dir, "B", "smem/x", "digest-brute")
    rf = bench.roofline(1e9, 0, 100.0)
    bench.attach_traffic(rf, "B", "smem/x", 100.0)
    assert rf["traffic"] == 1234560000
    assert rf["hbm_measured"]["achieved"] == pytest.approx(1234560000 / 0.1 / 1e9, rel=1e-3)

    for variant, digest in (("smem/y", "digest-brute"), ("smem/x", "stale")):
        write_profile(profile_dir, "B", variant, digest)
        rf = bench.roofline(1e9, 0, 100.0)
        bench.attach_traffic(rf, "B", "smem/x", 100.0)
        assert rf["traffic"] is None and "not attached" in rf["traffic_note"]

    # a BVH leg is matched against the BVH kernels' code digest
    write_profile(profile_dir, "C_bvh", "bvh4/x", "digest-bvh", hbm=99)
    rf = bench.roofline(1e6, 1e8, 50.0)
    bench.attach_traffic(rf, "C_bvh", "bvh4/x", 50.0)
    assert rf["traffic"] == 99


def test_frac_at_clock_from_the_profile(profile_dir):
    """A matrix-bound roofline is priced at the clock its PMC pass measured
    (VERDICT r4 item 2): peak x clock / 2.4 GHz, only for the digest-matched
    kernel; a VALU-bound leg carries no clock figures."""
    with open(profile_dir / "pmc_configB.json", "w") as f:
        json.dump({"config": "B", "kernel_variant": "mfmar/x", "kernel_source_sha256": "digest-brute",
                   "hbm_bytes_per_launch": 10, "clock_ghz": 1.92}, f)
    rf = bench.roofline(1.0214e12, 0, 160.0, 8.4e8, 1208, "mfmar/1024/k5/notn/res38/coop4/w4/cmp/cthr")
    assert rf["bound"] == "mfma"
    bench.attach_traffic(rf, "B", "mfmar/x", 160.0)
    assert rf["clock_ghz"] == 1.92
    assert rf["peak_at_clock"] == pytest.approx(rf["peak"] * 1.92 / 2.4, rel=1e-3)
    assert rf["frac_at_clock"] == pytest.approx(rf["frac"] * 2.4 / 1.92, rel=1e-3)
    rf = bench.roofline(1e9, 0, 100.0)  # the scalar path: VALU-bound
    bench.attach_traffic(rf, "B", "mfmar/x", 100.0)
    assert "frac_at_clock" not in rf


def test_roofline_figures():
    tests, kern_ms = 1.0214e12, 520.0
    rf = bench.roofline(tests, 0, kern_ms)
    flops = bench.FLOP_PER_TEST * tests / (kern_ms * 1e-3) / 1e12
    assert rf["achieved"] == pytest.approx(flops, rel=1e-3)
    assert rf["frac"] == pytest.approx(flops / bench.VALU_PEAK_TFLOPS, rel=1e-3)
    assert rf["bound"] == "valu" and rf["unit"] == "TFLOP/s" and rf["traffic"] is None
    assert "l2_read_algorithmic" not in rf  # brute force: no BVH gathers
    rf = bench.roofline(9e9, 3.77e11, 2900.0)
    l2 = (bench.BVH_RECORD_BYTES * 3.77e11 + bench.BVH_TRI_BYTES * 9e9) / 2.9 / 1e9
    assert rf["l2_read_algorithmic"]["achieved"] == pytest.approx(l2, rel=1e-3)
    assert rf["l2_read_algorithmic"]["peak"] == bench.L2_PEAK_GBS


def test_roofline_matrix_kernel():
    """render_mfma: matrix FLOP over the 16-padded triangle count of each
    segment against the dense F16 peak; the VALU-equivalent figure beside."""
    segs, n, kern_ms = 8.45e8, 1208, 417.0
    rf = bench.roofline(segs * n, 0, kern_ms, segs, n, "mfma/256/f16x3/coop16/w2")
    mf = bench.MFMA_FLOP_PER_PAIR * segs * 1216 / (kern_ms * 1e-3) / 1e12
    assert rf["bound"] == "mfma" and rf["peak"] == bench.MFMA_F16_PEAK_TFLOPS
    assert rf["achieved"] == pytest.approx(mf, rel=1e-3)
    assert rf["frac"] == pytest.approx(mf / bench.MFMA_F16_PEAK_TFLOPS, rel=1e-3)
    v = bench.FLOP_PER_TEST * segs * n / (kern_ms * 1e-3) / 1e12
    assert rf["valu_algorithmic"]["achieved"] == pytest.approx(v, rel=1e-3)
    # other kernels keep the VALU roofline even when given segments
    assert bench.roofline(segs * n, 0, kern_ms, segs, n, "smem/x")["bound"] == "valu"
    assert bench.kernel_label("mfma/256/f16x3/coop16/w2/imax").startswith("render_mfma")
    # the k16 sweep: 256 FLOP per pair over triangles padded to 32
    rf = bench.roofline(segs * n, 0, kern_ms, segs, n, "mfma/256/k16/coop8/w3/imax/minred/ymma/t12/llds/ser4/cmp")
    assert rf["achieved"] == pytest.approx(bench.MFMA_K16_FLOP_PER_PAIR * segs * 1216 / (kern_ms * 1e-3) / 1e12,
                                           rel=1e-3)
    # its 5-product form: 160 FLOP per pair
    rf = bench.roofline(segs * n, 0, kern_ms, segs, n, "mfma/256/k5/coop8/w3/imax/minred/ymma/t12/llds/ser4/cmp")
    assert rf["achieved"] == pytest.approx(bench.MFMA_K5_FLOP_PER_PAIR * segs * 1216 / (kern_ms * 1e-3) / 1e12,
                                           rel=1e-3)
    assert "5-product" in rf["flop_model"]
    rf = bench.roofline(segs * n, 0, kern_ms, segs, n, "mfma/256/k5/notn/coop8/w4/imax/minred/ymma/t12/llds2/ser4/cmp")
    assert rf["achieved"] == pytest.approx(bench.MFMA_K5_NOTN_FLOP_PER_PAIR * segs * 1216 / (kern_ms * 1e-3) / 1e12,
                                           rel=1e-3)


def test_kernel_labels():
    assert bench.kernel_label("assist12/max3f8/w6").startswith("render_assist")
    assert bench.kernel_label("bvh4/256/t16/w5").startswith("render_bvh4")
    assert bench.kernel_label("bvh3/256/t16/w5").startswith("render_bvh3")
    assert bench.kernel_label("smem/256/max3f8/coop32/w6/lockstep").startswith("render_smem")
    assert bench.kernel_label(None) is None


def _run_bench(args, env_extra=None, timeout=240):
    import subprocess
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=timeout)


def test_bench_gpus_flag_starts_its_own_ranks():
    """`bench.py --gpus 2` without a launcher starts 2 ranks itself (gloo here,
    --plumbing: the launch + row-tile gather path with no GPU) and reports
    n_gpus 2 with the gathered image checked on rank 0."""
    r = _run_bench(["--gpus", "2", "--no-cpu-baseline", "--plumbing", "--tile-rows", "3"],
                   {"RT2_BENCH_BACKEND": "gloo"})
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    assert lines[0]["n_gpus"] == 2 and lines[0]["gather_ok"] is True
    assert lines[0]["config"]["parallelism"] == "row-tile x2"


def test_bench_gpus_must_match_launcher_world():
    r = _run_bench(["--gpus", "4", "--plumbing"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr
