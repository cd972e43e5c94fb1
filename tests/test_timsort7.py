"""The oracle's JDK 7 Collections.sort (ComparableTimSort) restatement, used for
the reference's printed order on a Java 7 JVM (IntDocVectorsForwardIndex.java:
215, DocScore.compareTo at :363-365 = (int)Math.ceil(o.score - score)).

TimSort is not in the reference (a JDK class); the pins here are properties its
published algorithm must have:
  * on inputs where the DocScore comparator IS consistent (every score gap 0 or
    >= 1), ComparableTimSort is a stable sort: the result equals score desc, list
    order on ties (order 2) -- over run counts, galloping and both merge
    directions (lists up to 20,000, runs of every shape);
  * Java 6's legacy merge sort is the stable sort by score desc for ANY finite
    scores (it only asks compareTo <= 0 / > 0, tools/t5_divergence.py);
  * with gaps in (0, 1) the comparator is inconsistent: the two JVMs may then
    disagree, and TimSort either returns a permutation or throws (None).
"""
import numpy as np
import pytest

import oracle_lib as O


def _stable_desc(scores):
    return sorted(range(len(scores)), key=lambda i: (-scores[i], i))


@pytest.mark.parametrize("n", [0, 1, 2, 5, 31, 32, 33, 64, 100, 257, 1000, 4097, 20000])
def test_timsort_is_stable_on_consistent_inputs(n):
    g = np.random.default_rng(n)
    for trial in range(6):
        if trial == 0:
            s = g.integers(0, 5, size=n).astype(np.float64)          # many exact ties
        elif trial == 1:
            s = np.sort(g.integers(0, 40, size=n))[::-1].astype(np.float64)  # one descending run
        elif trial == 2:
            s = np.sort(g.integers(0, 40, size=n)).astype(np.float64)        # ascending: reversed runs
        elif trial == 3:  # runs of random lengths, alternating direction (galloping)
            parts, d = [], 1
            while sum(len(p) for p in parts) < n:
                m = int(g.integers(1, 300))
                parts.append(np.sort(g.integers(0, 1000, size=m))[::d])
                d = -d
            s = np.concatenate(parts)[:n].astype(np.float64) if parts else np.zeros(0)
        elif trial == 4:
            s = (g.integers(0, 3, size=n) * 2.0 + 0.5)                 # gaps of exactly 2
        else:
            s = g.integers(0, 10 ** 6, size=n).astype(np.float64)      # all distinct, gaps >= 1
        s = s.tolist()
        want = _stable_desc(s)
        assert O.sort_docscores(s, 3) == want, (n, trial)
        assert O.sort_docscores(s, 1) == want, (n, trial)


def test_legacy_merge_sort_is_stable_for_any_scores():
    g = np.random.default_rng(7)
    for n in (10, 100, 3000):
        s = (g.random(n) * 3).tolist()  # gaps in (0, 1) everywhere
        assert O.sort_docscores(s, 1) == _stable_desc(s)


def test_timsort_inconsistent_comparator():
    """Gaps below 1 compare 'equal' from one side: TimSort's `< 0` tests keep a
    higher score behind a lower one where it meets them in list order.  A short
    list (binary insertion only): [0.5, 1.2] -- compareTo(1.2, 0.5) = ceil(-0.7)
    = 0, not < 0, so 1.2 stays second; Java 6's merge sort asks compareTo(0.5,
    1.2) <= 0 -> ceil(0.7) = 1 > 0, so it swaps."""
    assert O.sort_docscores([0.5, 1.2], 3) == [0, 1]
    assert O.sort_docscores([0.5, 1.2], 1) == [1, 0]
    # longer lists: a permutation, or the contract-violation exception once a
    # merge runs out of its first run (dense gaps below 1 in long lists), never garbage
    g = np.random.default_rng(3)
    outcomes = set()
    for n, scale in ((64, 40.0), (300, 40.0), (5000, 4.0)):
        for trial in range(10):
            s = (g.random(n) * scale).tolist()
            p = O.sort_docscores(s, 3)
            outcomes.add(p is None)
            if p is not None:
                assert sorted(p) == list(range(n))
    assert outcomes == {True, False}
