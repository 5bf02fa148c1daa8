"""CPU: bench.py's multi-rank launch contract (no GPU needed).

* `bench.py --gpus 2` without WORLD_SIZE spawns two ranks itself (torch.distributed.run child,
  started before anything touches a GPU) and rank 0 prints ONE JSON line with n_gpus == 2;
* a rank refuses (exit 2) when WORLD_SIZE != --gpus;
* with fewer visible devices than ranks (here: none) the ranks refuse instead of sharing a GPU.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    e.update(kw)
    return e


def test_two_rank_rehearsal_prints_one_line_with_n_gpus_2():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--workload", "rehearse", "--steps", "3", "--warmup", "1"],
                       capture_output=True, text=True, timeout=240, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 3 and out["warmup"] == 1
    assert out["value"] > 0 and "rehearsal" in out
    # the shared-window sub-record: the keys the GPU line carries, from the
    # same sub_shared code path over gloo
    sh = out["shared"]
    for k in ("workload", "n_ranks", "scaling", "value", "unit", "steps", "ms_per_step", "plan_create_ms",
              "allreduce_ms_per_iteration", "allreduce_launches_per_iteration", "roofline", "config", "check"):
        assert k in sh, k
    assert sh["n_ranks"] == 2 and sh["scaling"] == "strong" and sh["allreduce_launches_per_iteration"] == 3
    assert sh["value"] > 0 and sh["allreduce_ms_per_iteration"] > 0


def test_world_size_mismatch_refused():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--workload", "rehearse"],
                       capture_output=True, text=True, timeout=120, env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr


def test_more_ranks_than_devices_refused():
    # this container has no GPU: every rank must refuse rather than share a device
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1", "--warmup", "0"],
                       capture_output=True, text=True, timeout=240, env=_env())
    assert r.returncode != 0
    assert "ranks never share a GPU" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
