"""bench.py's multi-rank path on the CPU: ``--gpus 2`` without torchrun launches two ranks
itself (gpmpc/launch.py), the ranks own contiguous instance shards, and the reported time is the
max over ranks (the driver runs ``bench.py --gpus N`` on one node)."""

import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _run(args):
    env = dict(os.environ, GPMPC_DIST_BACKEND="gloo", OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True, env=env,
                       timeout=240, cwd=str(ROOT))
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, p.stdout   # rank 0 prints exactly one line
    return json.loads(lines[0])


def test_self_launch_two_ranks_shards_and_max_timing():
    B, steps = 8, 6
    out = _run(["--gpus", "2", "--dry-run", "--batch", str(B), "--steps", str(steps), "--warmup", "1"])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 2 * B
    shards = out["shards"]
    assert [s[:2] for s in shards] == [[0, B], [B, 2 * B]]          # contiguous, disjoint, covering
    # rank r sleeps (1 + r) ms per step: the job time is the slowest rank's, not rank 0's
    slowest = max(s[2] for s in shards)
    assert slowest >= steps * 2e-3
    assert out["ms_per_step"] * 1e-3 * steps >= slowest - 1e-9
    assert abs(out["value"] - 2 * B * steps / (out["ms_per_step"] * 1e-3 * steps)) <= 1e-6 * out["value"]


def test_global_batch_strong_scaling_slices():
    """--global-batch G: contiguous B/G slices (sizes differing by at most one) covering every
    instance once; the job value counts G instances, scaling "strong"."""
    G, steps = 9, 4
    out = _run(["--gpus", "2", "--dry-run", "--global-batch", str(G), "--steps", str(steps), "--warmup", "0"])
    assert out["scaling"] == "strong" and out["config"]["global_batch"] == G
    assert [s[:2] for s in out["shards"]] == [[0, 5], [5, 9]]
    assert abs(out["value"] - G * steps / (out["ms_per_step"] * 1e-3 * steps)) <= 1e-6 * out["value"]
    sys.path.insert(0, str(ROOT / "gp-mpc_amd"))
    from gpmpc import distributed as D

    for g, w in ((1024, 8), (1024, 3), (7, 7), (100, 6)):
        sl = [D.shard_slice(g, r, w) for r in range(w)]
        assert sl[0].start == 0 and sl[-1].stop == g
        assert all(a.stop == b.start for a, b in zip(sl, sl[1:]))
        assert max(len(x) for x in sl) - min(len(x) for x in sl) <= 1


def test_default_partition_is_the_metrics_global_batch():
    """Without --batch, --gpus N splits the metric's global batch 1024 over the N ranks (strong
    scaling: the driver's SCALE runs measure "batch 1024 @1/2/4/8 GPU"), and the line carries the
    weak per-GPU figure (1024 instances on every GPU) as a secondary field."""
    out = _run(["--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "0"])
    assert out["scaling"] == "strong" and out["config"]["global_batch"] == 1024
    assert out["config"]["batch_per_gpu"] == 512
    assert [s[:2] for s in out["shards"]] == [[0, 512], [512, 1024]]
    w = out["weak_per_gpu"]
    assert w["scaling"] == "weak" and w["batch_per_gpu"] == 1024
    assert [s[:2] for s in w["shards"]] == [[0, 1024], [1024, 2048]]
    assert abs(w["value"] - 2048 * 3 / (w["ms_per_step"] * 3e-3)) <= 1e-6 * w["value"]
    one = _run(["--gpus", "1", "--dry-run", "--steps", "2", "--warmup", "0"])
    assert one["scaling"] == "strong" and one["config"]["global_batch"] == 1024 and one["weak_per_gpu"] is None
    assert one["shards"][0][:2] == [0, 1024]


def test_single_rank_needs_no_launcher():
    out = _run(["--gpus", "1", "--dry-run", "--batch", "4", "--steps", "2", "--warmup", "0"])
    assert out["n_gpus"] == 1 and out["shards"] == [[0, 4, out["shards"][0][2]]]


def _gpu_bench(args):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True, env=env,
                       timeout=240, cwd=str(ROOT))
    if p.returncode != 0 and "no GPU" in p.stderr:
        pytest.skip("no GPU")
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])



@pytest.mark.gpu
def test_bench_line_contract_on_the_gpu():
    """The driver's bench line on a short run: the contract keys, the roofline and
    cpu_baseline objects, the per-step kernel times and solver statistics are present and
    consistent (value = instances x steps / time, every instance-step converged)."""
    out = _gpu_bench(["--gpus", "1", "--steps", "3", "--warmup", "1", "--batch", "64", "--cpu-seconds", "1"])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in out, k
    assert out["steps"] == 3 and out["n_gpus"] == 1 and out["dtype"] == "f64" and out["scaling"] == "weak"
    assert abs(out["value"] - 64 * 3 / (out["ms_per_step"] * 3e-3)) <= 1e-6 * out["value"]
    r = out["roofline"]
    assert r["bound"] in ("hbm", "mfma") and r["unit"] == "TFLOP/s" and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-12
    # SURVEY 8(d)'s count with K_sqp = sqp_iter_mean, over the launch; the executed count beside it
    assert abs(r["flops_per_launch"] - 64 * out["sqp_iter_mean"] * 480_000) <= 1e-9 * r["flops_per_launch"]
    assert 0.0 < r["executed"]["achieved"] and r["regime"] == "latency"
    lat = r["latency"]   # per-instance solve time (s_memrealtime) against the kernel's
    assert 0.0 < lat["mean_instance_ms_per_step"] <= lat["slowest_instance_ms_per_step"]
    assert 0.3 < lat["slowest_over_kernel"] <= 1.05, lat
    assert out["build"]["matches_tree"], out["build"]
    assert len(out["sqp_kernel_ms_per_step_distribution"]["per_step"]) == 3
    assert out["status_counts"]["0"] == 64 * 3
    assert 1.0 <= out["linearisations_per_step"] <= out["sqp_iter_mean"] + 1.0
    cb = out["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] in ("port", "reference")
    assert cb["window"] == [1, 4] and cb["sqp_iter_mean"] > 0   # the GPU leg's own timed window


def test_flop_counts_match_survey_8d():
    """bench.py's roofline flop counts for config 3 (quad2d, N=200, H=30): the executed count
    evaluates the u-only thrust GP once per stage, SURVEY.md 8(d)'s count at all 4 RK4 points;
    per linearisation and GP, 2d + 2(d+1) flops per training point and evaluation; the exact
    variance costs N(N+1) + 2N per stage and GP."""
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "gp-mpc_amd"))
    import bench
    from gpmpc.models import get_spec

    spec = get_spec("quad2d")
    H, N = 30, 200
    per_lin, exps_lin, var = bench.gp_flops(spec, N, H)
    thrust, pitch = 2 * 1 + 2 * 2, 2 * 3 + 2 * 4          # d = 1 (T_c) and d = 3 (theta, theta_dot, P_c)
    assert sorted(spec.gp_dims) == [1, 3]
    assert per_lin == H * N * (thrust + 4 * pitch) == 372_000
    assert bench.survey_flops_per_lin(spec, N, H) == H * 4 * N * (thrust + pitch) == 480_000
    assert exps_lin == H * N * (1 + 4)
    assert var == 2 * H * (N * (N + 1) + 2 * N)


def test_shard_mode_runs_one_rank_alone():
    """--shard R/N measures one rank of an N-rank strong-scaled job by itself (tools/shard_sweep.sh):
    it is a single process on the GPU, so it refuses a process group and the CPU rehearsal."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--shard", "1/2", "--dry-run", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=240, cwd=str(ROOT))
    assert p.returncode != 0 and "--shard R/N runs one rank alone" in p.stderr
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--shard", "2/2", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=240, cwd=str(ROOT))
    assert p.returncode != 0 and "0 <= R < N" in p.stderr


@pytest.mark.gpu
def test_emulated_shard_line_on_the_gpu():
    """Every rank's shard reports its own line (rank > 0 included): its slice of the metric's global
    batch, value = the shard's instances x steps / its time, no CPU baseline."""
    out = _gpu_bench(["--shard", "3/8", "--steps", "2", "--warmup", "1"])
    assert out["emulated_shard"]["rank"] == 3 and out["emulated_shard"]["world"] == 8
    assert out["emulated_shard"]["instances"] == [384, 512] and out["config"]["batch_per_gpu"] == 128
    assert out["cpu_baseline"] is None and out["scaling"] == "strong"
    assert abs(out["value"] - 128 * 2 / (out["ms_per_step"] * 2e-3)) <= 1e-6 * out["value"]
    assert sum(out["status_counts"].values()) == 128 * 2
    # the shard's statistics are normalised by its own instances (no all-reduce in shard mode)
    assert out["sqp_iter_mean"] >= 1.0 and out["linearisations_per_step"] >= 1.0
