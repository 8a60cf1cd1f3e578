"""bench.py's launcher (CPU): `--gpus N` without a torchrun environment starts N ranks under
torch.distributed.run (127.0.0.1), every rank sees world size N, and exactly one JSON line
comes from rank 0 -- the driver's multi-GPU contract, rehearsed on gloo."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    res = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args,
                         capture_output=True, text=True, timeout=240, env=env)
    assert res.returncode == 0, res.stdout + res.stderr
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    return [json.loads(ln) for ln in lines]


def test_gpus_flag_spawns_ranks():
    out = _run(["--gpus", "2", "--dry-run"])
    assert len(out) == 1 and out[0]["n_gpus"] == 2 and out[0]["rank"] == 0


def test_gpus8_reaches_rccl_init():
    """--gpus 8: eight ranks each run the real path's RCCL initialisation (bench.init_rccl:
    init_process_group("nccl", device_id=cuda:LOCAL_RANK)); with no GPU here each stops at the
    device_id check for its own local rank, after the argument parsing and the launcher's
    environment were accepted.  Rank 0 reports all eight."""
    import pytest
    import torch
    n_dev = torch.cuda.device_count()
    if 0 < n_dev < 8:
        # ranks without a device fail their RCCL init while the others wait in its rendezvous
        pytest.skip(f"{n_dev} GPU(s): the 8-rank RCCL rehearsal needs 0 (CPU) or >= 8")
    out = _run(["--gpus", "8", "--dry-run", "nccl"])
    assert len(out) == 1 and out[0]["n_gpus"] == 8 and out[0]["backend"] == "nccl"
    ranks = out[0]["ranks"]
    assert [r["rank"] for r in ranks] == list(range(8))
    assert [r["local_rank"] for r in ranks] == list(range(8))
    for r in ranks:
        if n_dev == 0:
            assert r["nccl"].startswith("device_id check") and f"cuda:{r['local_rank']}" in r["nccl"]
        else:
            assert r["nccl"].startswith("rccl initialised")


def test_single_rank_default():
    out = _run(["--dry-run"])
    assert len(out) == 1 and out[0]["n_gpus"] == 1


def test_world_mismatch_fails():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    res = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                          "--dry-run"], capture_output=True, text=True, timeout=120, env=env)
    assert res.returncode != 0 and "WORLD_SIZE" in (res.stdout + res.stderr)


def test_leg_watchdog_prints_line_and_exits():
    """A multi-rank side leg that never returns (e.g. a collective whose peer failed) must not
    lose the metric line: the watchdog prints it with the pending legs marked, then exits
    non-zero (bench.LEG_STALL_EXIT) so the stall reads as a failure to the launcher."""
    import json
    import subprocess
    import sys
    code = ("import sys, time; sys.path.insert(0, %r); import bench; "
            "bench.LEG_DEADLINE_S = 0.5; "
            "bench._LegWatchdog({'value': 1.0, 'c3_small_blobs': {'encode_gibs': 2.0}, "
            "'c4_partitioned': None}, 0, 0.5); time.sleep(30)") % ROOT
    res = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=20)
    assert res.returncode == 3, (res.returncode, res.stderr[-500:])
    assert "stalled" in res.stderr
    line = json.loads(res.stdout.strip().splitlines()[-1])
    assert line["value"] == 1.0 and line["c3_small_blobs"] == {"encode_gibs": 2.0}
    assert "not finished" in line["c4_partitioned"]["error"]
