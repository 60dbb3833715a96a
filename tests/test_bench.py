"""bench.py's bookkeeping on CPU: the PMC profile is used only for the build it was measured on,
the CPU baseline's core count, the algorithmic byte counts of SURVEY.md §8(d)."""
import json
import os

import bench


def test_pmc_profile_only_for_the_build_it_was_measured_on(tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    entry = {"hbm_bytes_per_launch": 1.0, "profile": "rX", "so_sha16": "0" * 16}
    (prof / "pmc_traffic.json").write_text(json.dumps({"config4_f64": entry}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "lib_sha16", lambda: "f" * 16)
    pmc, note = bench.read_pmc("f64", 4)
    assert pmc is None and "another build" in note
    monkeypatch.setattr(bench, "lib_sha16", lambda: "0" * 16)
    pmc, note = bench.read_pmc("f64", 4)
    assert pmc == entry and "rX" in note
    pmc, note = bench.read_pmc("f32", 4)
    assert pmc is None and "no PMC profile" in note


def test_host_threads_honours_the_granted_share(monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "16")
    assert bench.host_threads() == 16
    monkeypatch.delenv("OMP_NUM_THREADS")
    assert bench.host_threads() == (os.cpu_count() or 1)


def test_algorithmic_bytes_per_vehicle():
    # f64: 11 reals + 3 int32 + 4 uint8 read, 10 reals + 3 int32 + 2 uint8 written (one fused launch)
    assert bench.state_bytes("f64") == (11 * 8 + 12 + 4, 10 * 8 + 12 + 2)
    assert bench.state_bytes("f32") == (11 * 4 + 12 + 4, 10 * 4 + 12 + 2)


def test_configs_match_baseline_json():
    base = json.load(open(os.path.join(bench.ROOT, "BASELINE.json")))
    assert len(base["configs"]) == 5
    assert (bench.CONFIGS[4]["num_envs"], bench.CONFIGS[4]["vehicles"]) == (4096, 64)
    assert (bench.CONFIGS[2]["num_envs"], bench.CONFIGS[2]["vehicles"]) == (4096, 32)
    assert (bench.CONFIGS[3]["num_envs"], bench.CONFIGS[3]["vehicles"]) == (4096, 128)
    assert (bench.CONFIGS[5]["num_envs"], bench.CONFIGS[5]["vehicles"]) == (8192, 64)
    assert (bench.CONFIGS[1]["num_envs"], bench.CONFIGS[1]["vehicles"]) == (1, 50)
    assert bench.CONFIGS[3]["obs"]["type"] == "OccupancyGrid"


def _run_bench(*argv, env_extra=None):
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(bench.ROOT, "bench.py"), *argv], capture_output=True,
                       text=True, env=env, timeout=240)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p.stderr


def test_gpus_n_runs_n_ranks_from_a_plain_invocation():
    """`python bench.py --gpus 2` (how the driver may call it) runs a 2-rank torch.distributed.run
    child job; the parent imports no torch (so it opens no device) and relays rank 0's line, which
    reports n_gpus == 2 with the weak-scaling shards [r*E, (r+1)*E)."""
    rc, out, err = _run_bench("--gpus", "2", "--dry-run")
    assert rc == 0, err
    assert out["n_gpus"] == 2 and out["scaling"] == "weak"
    assert [tuple(s) for s in out["shards"]] == [(0, 4096), (4096, 4096)]
    assert out["launcher"]["ranks"] == 2 and out["launcher"]["parent_imported_torch"] is False
    assert out["max_elapsed"] == 0.002  # the max over both ranks


def test_strong_scaling_splits_the_global_batch():
    rc, out, err = _run_bench("--gpus", "2", "--dry-run", "--strong")
    assert rc == 0, err
    assert out["scaling"] == "strong" and out["global_envs"] == 32768
    assert [tuple(s) for s in out["shards"]] == [(0, 16384), (16384, 16384)]
    rc, out, err = _run_bench("--gpus", "1", "--dry-run", "--strong", "--global-envs", "1000")
    assert rc == 0 and out["n_gpus"] == 1 and [tuple(s) for s in out["shards"]] == [(0, 1000)]


def test_world_size_must_equal_gpus():
    rc, out, err = _run_bench("--gpus", "2", "--dry-run", env_extra={"WORLD_SIZE": "1"})
    assert rc == 2 and "WORLD_SIZE=1" in err
