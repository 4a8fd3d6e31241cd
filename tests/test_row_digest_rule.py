"""The one-chunk row-digest rule.

Winterfell's RowMatrix::commit_to_rows hashes a row with hash_elements when partition_size ==
num_cols and otherwise with merge_many over the chunk digests, even when the row forms a single
chunk [WF-recall]; the reference's own restatement hash_row_poseidon (agg/child.rs:1025-1045)
returns a single chunk digest as is.  The two rules differ ONLY on rows narrower than their
partition size: the 7-column composition rows once select_partitions_for_trace (utils.rs:
394-409) returns 2 or more partitions (n >= 2^14), and any matrix narrower than hash_rate.
Both oracle and library carry the rule as one named switch (default 0 = Winterfell)."""
import random

import pytest


@pytest.fixture
def rule(oracle):
    yield oracle.set_row_digest_rule
    oracle.set_row_digest_rule(0)


@pytest.mark.parametrize("ncols,np_,rate", [
    (204, 1, 16), (204, 2, 16), (204, 4, 16), (204, 16, 16),   # trace rows: 1 or several chunks
    (219, 4, 16), (211, 8, 16),
    (7, 1, 16),                                                  # composition rows below 2^14 rows
    (7, 2, 16), (7, 4, 16), (7, 16, 16),                         # composition rows from 2^14 rows up
    (31, 1, 8), (31, 2, 8), (16, 2, 16), (17, 2, 16), (33, 2, 16),
])
def test_rules_differ_only_on_one_chunk_rows(oracle, rule, ncols, np_, rate):
    rng = random.Random(ncols * 131 + np_)
    row = [rng.randrange(oracle.P) for _ in range(ncols)]
    ps = oracle.partition_size(np_, rate, ncols)
    chunks = -(-ncols // ps)
    d0 = oracle.row_digest(row, ps)
    rule(1)
    d1 = oracle.row_digest(row, ps)
    one_chunk_partitioned = ps != ncols and chunks == 1
    assert (d0 != d1) == one_chunk_partitioned
    # rule 0 is Winterfell's commit_to_rows, rule 1 agg/child.rs hash_row_poseidon
    if ps == ncols:
        assert d0 == oracle.hash_elements(row)
    else:
        digs = [oracle.hash_elements(row[c:c + ps]) for c in range(0, ncols, ps)]
        assert d0 == oracle.merge_many(digs)
        assert d1 == (digs[0] if chunks == 1 else oracle.merge_many(digs))


def test_headline_rows_affected(oracle):
    """At the headline shape (n = 2^16: 4 partitions, rate 16) the trace rows (204 columns,
    4 chunks of 51) hash the same under both rules, the composition rows (7 columns, partition
    size 16, one chunk) do not; below 2^14 rows (1 partition) nothing differs."""
    for n, w, c in [(1 << 16, 204, 7), (1 << 14, 204, 7), (1 << 13, 204, 7), (1 << 20, 219, 7)]:
        np_ = 16 if n >= 1 << 20 else 8 if n >= 1 << 18 else 4 if n >= 1 << 16 else 2 if n >= 1 << 14 else 1
        tps, cps = oracle.partition_size(np_, 16, w), oracle.partition_size(np_, 16, c)
        assert -(-w // tps) > 1 or tps == w
        assert (cps != c) == (n >= 1 << 14)


def test_proofs_differ_exactly_in_the_composition_commitment(oracle, rule):
    """A 2^6-row segment proved with partitions (2, 16): trace rows form two chunks, composition
    rows one.  The two rules give different proofs, each verifies under its own rule, and a
    proof checked under the other rule fails at the constraint (composition) Merkle opening —
    after the trace opening has been accepted — so the composition row digests are the only
    difference."""
    t, pi, w = oracle.synth_segment(0x5EED0A06, 6)
    opts = oracle.default_options(w, 64, queries=12, grind=2)
    opts.num_partitions = 2
    p0 = oracle.prove(t, w, 64, pi, opts)
    assert oracle.verify(p0, pi, opts)[0] == 0
    rule(1)
    p1 = oracle.prove(t, w, 64, pi, opts)
    assert p1 != p0
    assert oracle.verify(p1, pi, opts)[0] == 0
    rc, err = oracle.verify(p0, pi, opts)
    assert rc != 0 and "constraint Merkle opening" in err
    rule(0)
    rc, err = oracle.verify(p1, pi, opts)
    assert rc != 0 and "constraint Merkle opening" in err
    # one partition: both rules give the same proof
    opts.num_partitions = 1
    a = oracle.prove(t, w, 64, pi, opts)
    rule(1)
    assert oracle.prove(t, w, 64, pi, opts) == a
