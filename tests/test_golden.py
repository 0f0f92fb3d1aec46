"""Golden vectors (tests/golden/topics_golden.json, made by tests/golden/make_golden.py from the
oracle after it passes the reference's known-answer tests): the oracle must still produce them
(CPU), and the HIP engine must produce them bit-exactly through the C-ABI (GPU)."""
import json
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
from make_golden import jsonable, replay  # noqa: E402

from adapters import EngineAdapter, OracleAdapter  # noqa: E402


@pytest.fixture(scope="module")
def golden():
    with open(os.path.join(HERE, "golden", "topics_golden.json")) as f:
        return json.load(f)


def _check(ix, g, batch=False):
    assert replay(ix, g["ops"]) == g["returns"]
    got = ix.subscribers_batch(g["topics"]) if batch else [ix.subscribers(t) for t in g["topics"]]
    for t, s, want in zip(g["topics"], got, g["subscribers"]):
        assert jsonable(s) == want, t
    msgs = ix.messages_batch(g["filters"]) if batch else [ix.messages(f) for f in g["filters"]]
    for f, m, want in zip(g["filters"], msgs, g["messages"]):
        assert sorted(int(h) for h in m) == want, f


def test_oracle_reproduces_golden(golden):
    _check(OracleAdapter(), golden)


@pytest.mark.gpu
def test_engine_matches_golden(golden, gpu_available):
    _check(EngineAdapter(), golden, batch=True)
