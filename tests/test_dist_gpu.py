"""The N>1 libsme path on one GPU: two fresh rank processes (gloo collectives)
each build a shard with libsme (cuts from sme_split_points), all-reduce N and
df -- keyed by device term fingerprints -- into sme_index_reweight, score, and
merge the per-shard top-k lists; the result must equal the single-index oracle
bit for bit in both idf modes, for top-10 and top-100."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("idf_mode", [0, 1])
def test_two_libsme_shards(tmp_path, idf_mode):
    worker = os.path.join(os.path.dirname(__file__), "dist_gpu_worker.py")
    port = str(_free_port())
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    procs = [subprocess.Popen([sys.executable, worker, str(r), "2", port, str(idf_mode), str(tmp_path)], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(2)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out.decode(errors="replace")[-3000:])
    assert all(p.returncode == 0 for p in procs), outs
    assert (tmp_path / "ok0").exists() and (tmp_path / "ok1").exists()
