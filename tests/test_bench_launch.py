"""bench.py's launch decision (CPU): `--gpus N` runs N ranks, one process per
GPU, whether the driver launches them (torch.distributed.run sets WORLD_SIZE)
or bench.py is started bare; a WORLD_SIZE that disagrees with --gpus fails.
Also the cgroup-aware CPU count the cpu_baseline reports."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_one_gpu_runs_in_process():
    assert bench.launch_plan(1, {}) == "rank"


def test_n_gpus_without_world_spawns():
    for n in (2, 4, 8):
        assert bench.launch_plan(n, {}) == "spawn"


def test_driver_launch_is_a_rank():
    for n in (1, 2, 8):
        assert bench.launch_plan(n, {"WORLD_SIZE": str(n)}) == "rank"


def test_world_mismatch_fails():
    with pytest.raises(SystemExit) as e:
        bench.launch_plan(8, {"WORLD_SIZE": "1"})
    assert "WORLD_SIZE=1" in str(e.value)
    with pytest.raises(SystemExit):
        bench.launch_plan(1, {"WORLD_SIZE": "2"})
    with pytest.raises(SystemExit):
        bench.launch_plan(0, {})


def test_spawn_command(monkeypatch):
    seen = {}

    class Done:
        returncode = 7

    def fake_run(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return Done()

    monkeypatch.setattr(subprocess, "run", fake_run)
    rc = bench.spawn_ranks(4, ["--gpus", "4", "--config", "4"])
    assert rc == 7
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert int(cmd[cmd.index("--master-port") + 1]) > 0
    assert cmd[-5:] == [os.path.join(ROOT, "bench.py"), "--gpus", "4", "--config", "4"]


@pytest.mark.timeout(180)
def test_bare_gpus2_starts_two_ranks_and_propagates_failure():
    """No GPU here: each of the two spawned ranks must get as far as its
    device check and fail loudly; the parent exits non-zero (it never reports
    a one-GPU number for --gpus 2)."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("LCFIR_BENCH_SHARE_DEVICE", None)
    env["HIP_VISIBLE_DEVICES"] = ""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                         cwd=ROOT, capture_output=True, text=True, timeout=170, env=env)
    assert out.returncode != 0
    text = out.stdout + out.stderr
    assert "rank 0 needs GPU 0" in text and "rank 1 needs GPU 1" in text, text[-3000:]
    assert not any(l.startswith("{") for l in out.stdout.splitlines())


def test_usable_cpus_reads_cgroup_quota(tmp_path):
    (tmp_path / "cpu.max").write_text("1600000 100000\n")
    usable, aff, quota = bench.usable_cpus(str(tmp_path))
    assert quota == 16 and aff == bench.host_cores() and usable == min(aff, 16)
    (tmp_path / "cpu.max").write_text("max 100000\n")
    usable, aff, quota = bench.usable_cpus(str(tmp_path))
    assert quota is None and usable == aff
    (tmp_path / "cpu.max").write_text("150000 100000\n")  # 1.5 CPUs -> 2 threads
    assert bench.cgroup_cpu_quota(str(tmp_path)) == 2


def test_usable_cpus_cgroup_v1(tmp_path):
    (tmp_path / "cpu").mkdir()
    (tmp_path / "cpu" / "cpu.cfs_quota_us").write_text("800000\n")
    (tmp_path / "cpu" / "cpu.cfs_period_us").write_text("100000\n")
    assert bench.cgroup_cpu_quota(str(tmp_path)) == 8
    (tmp_path / "cpu" / "cpu.cfs_quota_us").write_text("-1\n")
    assert bench.cgroup_cpu_quota(str(tmp_path)) is None
    assert bench.cgroup_cpu_quota(str(tmp_path / "missing")) is None


def test_rank_spread_reduction():
    """The N > 1 line's per-rank block: lists in rank order, min and max of
    each figure (value and ms_per_step stay max-based)."""
    recs = [{"rank": 0, "device": "0000:05:00 (cuda:0)", "ms_per_step": 1.30, "kernel_ms": 1.10,
             "allreduce_ms_per_step": 0.05, "samples": 10},
            {"rank": 1, "device": "0000:15:00 (cuda:1)", "ms_per_step": 1.45, "kernel_ms": 1.12,
             "allreduce_ms_per_step": 0.21, "samples": 10}]
    r = bench.rank_spread(recs)
    assert r["rank"] == [0, 1] and r["device"] == ["0000:05:00 (cuda:0)", "0000:15:00 (cuda:1)"]
    assert r["ms_per_step"] == [1.30, 1.45] and r["ms_per_step_min"] == 1.30 and r["ms_per_step_max"] == 1.45
    assert r["kernel_ms_max"] == 1.12 and r["allreduce_ms_per_step_min"] == 0.05
    # no exchange on the step: the all-reduce fields are null, not 0
    recs = [dict(d, allreduce_ms_per_step=None) for d in recs]
    r = bench.rank_spread(recs)
    assert r["allreduce_ms_per_step"] == [None, None] and r["allreduce_ms_per_step_max"] is None


def _gather_worker(rank, world):
    import torch.distributed as dist
    mine = {"rank": rank, "device": f"cpu{rank}", "ms_per_step": 1.0 + rank, "kernel_ms": 0.5,
            "allreduce_ms_per_step": 0.1 * (rank + 1), "samples": 100 * (rank + 1)}
    records = [None] * world
    dist.all_gather_object(records, mine)
    return bench.rank_spread(records) if rank == 0 else None


@pytest.mark.timeout(120)
def test_rank_spread_gathered_over_gloo():
    """bench.py's all_gather_object of the per-rank records, world 2 on gloo."""
    import gloo_ranks
    r = gloo_ranks.run(_gather_worker, 2, timeout=100)[0]
    assert r["rank"] == [0, 1] and r["device"] == ["cpu0", "cpu1"]
    assert r["ms_per_step_max"] == 2.0 and r["samples"] == [100, 200]
    assert r["allreduce_ms_per_step_max"] == pytest.approx(0.2)
