"""Generates tests/golden/*.json from the pure-Python restatement (tests/pyref.py).
Run: python tests/golden/make_golden.py"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import pyref  # noqa: E402

P = pyref.P
inp = [(i * 0x9E3779B97F4A7C15 * 0x1234567) % P for i in range(1, 52)]
a, b = inp[3], inp[7]
out = {
    "hash_elements": {"input": inp, "output": pyref.hash_elements(inp)},
    "merge": {"input": [a, b], "output": pyref.merge(a, b)},
    "merge_with_int": {"input": [a, 65536], "output": pyref.merge_with_int(a, 65536)},
    "hasher_dom": pyref.hasher_suite()[0],
}
json.dump(out, open(os.path.join(HERE, "poseidon_vectors.json"), "w"), indent=1)
print("wrote poseidon_vectors.json")
