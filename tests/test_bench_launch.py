"""bench.py's launch contract: `--gpus N` must run N ranks and say so.

The driver runs `bench.py --gpus N` either under torch.distributed.run (WORLD_SIZE
set) or directly; directly, bench.py starts the N rank processes itself.  The
world size the ranks agree on must equal --gpus, so an N-GPU line cannot
silently measure one GPU.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def test_gpus_mismatch_refused():
    """WORLD_SIZE from a launcher that disagrees with --gpus: refused before any
    GPU work (no torch import on this path)."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "--gpus 2 but WORLD_SIZE=1" in (r.stderr + r.stdout)


@pytest.mark.gpu
def test_gpus2_rehearsal_spawns_two_ranks():
    """`bench.py --gpus 2` with no launcher, rehearsed on one GPU
    (SME_BENCH_REHEARSE=1: two ranks share the device, gloo collectives): the
    line says n_gpus 2 and every full-size check of the sharded run holds."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["SME_BENCH_REHEARSE"] = "1"
    cmd = [sys.executable, BENCH, "--gpus", "2", "--docs", "2000", "--queries", "200", "--steps", "1", "--warmup",
           "1", "--cpu-docs", "0", "--no-e2e"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, r.stdout[-2000:]
    d = json.loads(line[0])
    assert d["n_gpus"] == 2 and "rehearsal" in d
    assert d["config"]["docs_this_gpu"] == 2000
    assert d["query"]["queries"] == 200
    bad = [k for k, v in d["checks"].items() if v is False]
    assert not bad, bad
