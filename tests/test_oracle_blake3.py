"""BLAKE3 known answers (published spec test vectors; input byte i = i % 251)."""
import os

import pytest

KAT = {
    b"": "af1349b9f5f9a1a6a0404dea36dcc9499bcb25c9adc112b7cc9a93cae41f3262",
    b"abc": "6437b3ac38465133ffb63b75273a8db548c558465d79db03fd359c6cd5bd9d85",
}
# prefixes of the official test_vectors.json hashes (hash mode)
SPEC_PREFIX = {
    1: "2d3adedff11b61f14c886e35afa03673",
    1024: "42214739f095a406f3fc83deb889744a",
    1025: "d00278ae47eb27b34faecf67b4fe263f",
    2048: "e776b6028c7cd22a4d0ba182a8bf6220",
}


def test_kat(oracle):
    for msg, h in KAT.items():
        assert oracle.blake3(msg).hex() == h


def test_spec_vectors(oracle):
    for n, pre in SPEC_PREFIX.items():
        assert oracle.blake3(bytes(i % 251 for i in range(n))).hex().startswith(pre)


def test_matches_python_restatement(oracle):
    import pyref
    for n in (0, 1, 63, 64, 65, 1023, 1024, 1025, 2049, 5000):
        msg = bytes((i * 13 + 5) % 256 for i in range(n))
        assert oracle.blake3(msg) == pyref.blake3(msg)


def test_rollup_bench_commitment_note(oracle):
    """BASELINE.md's program commitment (0x07d8a570...) was printed from a 2025-11-24 run;
    the example file in the 2025-12-26 snapshot hashes differently, so it cannot pin BLAKE3.
    Only checked when the reference tree is present (never on the GPU box)."""
    path = "/root/reference/examples/rollup-bench.zlisp"
    if not os.path.exists(path):
        pytest.skip("reference tree not present")
    src = open(path, "rb").read()
    import pyref
    assert oracle.blake3(src) == pyref.blake3(src)
