"""The N>1 libsme path on one GPU: fresh rank processes (gloo collectives) each
build a shard with libsme (cuts from sme_split_points), all-reduce N and df --
keyed by device term fingerprints -- into sme_index_reweight, score, and merge
the per-shard top-k lists by query owner; the result must equal the
single-index oracle bit for bit in both idf modes, for top-10 and top-100.
Two ranks over a small corpus, and four ranks over the c4 distribution."""
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


def _run_ranks(script, world, args, tmp_path, timeout):
    worker = os.path.join(os.path.dirname(__file__), script)
    port = str(_free_port())
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    procs = [subprocess.Popen([sys.executable, worker, str(r), str(world), port] + args + [str(tmp_path)], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(world)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out.decode(errors="replace")[-3000:])
    assert all(p.returncode == 0 for p in procs), outs
    assert all((tmp_path / ("ok%d" % r)).exists() for r in range(world))


@pytest.mark.parametrize("idf_mode", [0, 1])
def test_two_libsme_shards(tmp_path, idf_mode):
    _run_ranks("dist_gpu_worker.py", 2, [str(idf_mode)], tmp_path, 240)


def test_c4_four_shards(tmp_path):
    """BASELINE config c4 (50M docs doc-sharded over GPUs with a df all-reduce),
    exercised through the multi-rank path at 60,000 docs of the c4 distribution
    (V_w = 2^22, 200-360 tokens, seed 44): four rank processes, each a libsme
    shard of a Hadoop split; fingerprint df exchange + reweight in both idf
    modes; 1,100 golden queries merged by query owner, equal to the
    single-index oracle bit for bit (tests/dist_c4_worker.py)."""
    import json
    _run_ranks("dist_c4_worker.py", 4, [], tmp_path, 400)
    t = [json.load(open(tmp_path / ("timing%d.json" % r))) for r in range(4)]
    assert sum(x["queries_checked"] for x in t) == 1100
    print("df exchange (rank 0, gloo):", json.dumps(t[0]["df_exchange_mode1"]))


@pytest.mark.parametrize("world", [2, 3])
def test_reference_partitions(tmp_path, world):
    """Reference-layout output from doc shards: the term-partition all_to_all of
    postings and the owners' per-term reducer merge give exactly the oracle's R
    part files for the same map tasks (R = 10 and 3), with docids duplicated
    across shards merged as the single reducer merges them
    (tests/dist_parts_worker.py)."""
    _run_ranks("dist_parts_worker.py", world, [], tmp_path, 240)


@pytest.mark.parametrize("K", [2, 3])
def test_reference_partitions_kgrams(tmp_path, K):
    """The same world-2 reference-layout exchange for a K-gram index: grams
    travel as their component terms joined by U+0000 (TermDF.compareTo order,
    Arrays.hashCode partitions over the components) and the owners' merged part
    files equal the oracle's K-gram job over the same two map tasks."""
    _run_ranks("dist_parts_worker.py", 2, [str(K)], tmp_path, 240)
