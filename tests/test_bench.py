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
