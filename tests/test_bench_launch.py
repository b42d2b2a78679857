"""bench.py's multi-GPU launch contract, on CPU: ``--gpus N`` without a launcher starts N rank
processes itself (fresh processes, RANK / WORLD_SIZE / MASTER_* set, 127.0.0.1 rendezvous), and a
launcher whose WORLD_SIZE differs from --gpus is refused before anything touches the GPU."""
import os
import subprocess
import sys
from pathlib import Path

import bench
import pytest

ROOT = Path(__file__).resolve().parents[1]


def test_check_world_matches():
    assert bench.check_world(1, {}) == (1, None)
    assert bench.check_world(4, {"WORLD_SIZE": "4"}) == (4, None)


def test_check_world_mismatch_fires():
    world, err = bench.check_world(8, {"WORLD_SIZE": "1"})
    assert world == 1 and "--gpus 8" in err
    _, err = bench.check_world(1, {"WORLD_SIZE": "2"})
    assert err is not None


def test_bench_refuses_mismatched_launcher():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=3" in r.stderr


def test_spawn_ranks_starts_n_processes(tmp_path):
    probe = tmp_path / "probe.py"
    out = tmp_path / "ranks"
    out.mkdir()
    probe.write_text(
        "import os, sys\n"
        "open(os.path.join(sys.argv[1], os.environ['RANK']), 'w').write(\n"
        "    ' '.join(os.environ[k] for k in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT')))\n")
    env_before = dict(os.environ)
    rc = bench.spawn_ranks(3, [str(out)], script=probe)
    assert rc == 0
    assert dict(os.environ) == env_before       # the parent's env is untouched
    seen = sorted(p.read_text().split() for p in out.iterdir())
    assert [s[:3] for s in seen] == [["0", "0", "3"], ["1", "1", "3"], ["2", "2", "3"]]
    assert {s[3] for s in seen} == {"127.0.0.1"} and len({s[4] for s in seen}) == 1


def test_spawn_ranks_reports_failure(tmp_path):
    probe = tmp_path / "fail.py"
    probe.write_text("import os, sys\nsys.exit(3 if os.environ['RANK'] == '1' else 0)\n")
    assert bench.spawn_ranks(2, [], script=probe) == 3


def test_spawn_ranks_stops_blocked_rank0_when_rank1_fails(tmp_path):
    """Rank 0 blocked (as in a collective on a dead peer) while rank 1 exits 3: spawn_ranks returns
    3 promptly and stops rank 0, instead of waiting on rank 0 first."""
    probe = tmp_path / "hang.py"
    probe.write_text("import os, sys, time\n"
                     "if os.environ['RANK'] == '1':\n"
                     "    sys.exit(3)\n"
                     "time.sleep(600)\n")
    t0 = __import__("time").perf_counter()
    assert bench.spawn_ranks(2, [], script=probe) == 3
    assert __import__("time").perf_counter() - t0 < 30


def test_headline_value_is_the_whole_step_at_n_gt_1():
    """N > 1: ``value`` comes from the gathered step (slice GEMM + all-gather, the full Y on every
    rank), never from the slice GEMM alone, which stays the side key ``kernel_only``."""
    h1 = bench.headline(1, 4096, 10, t_slice=1e-3)
    assert h1["value_from"] == "gemm" and h1["value"] == 4096 * 10 / 1e-3 and "kernel_only" not in h1
    h4 = bench.headline(4, 4096, 10, t_slice=0.4e-3, t_full=0.9e-3, chunks=2)
    assert h4["value"] == 4096 * 10 / 0.9e-3 and abs(h4["ms_per_step"] - 0.09) < 1e-12
    assert h4["value_from"].startswith("gemm+allgather")
    assert h4["kernel_only"]["value"] == round(4096 * 10 / 0.4e-3, 1)
    with pytest.raises(ValueError):
        bench.headline(2, 4096, 10, t_slice=1e-3)
