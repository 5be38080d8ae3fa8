"""Limits of the token representation (engine_common.h): an end code holds a
token span of at most END_MAX = 2^31 - 3 bytes.  A run of one byte merged by
doubling merges produces ever longer tokens; past the limit every path --
training (one-merge engine and batches), the global encode replay that long
runs fall back to -- must stop with BPE_GPU_ERANGE instead of writing a
wrong end code.  BPE_END_MAX lowers the limit so a 5000-byte run reaches it."""
import os

import numpy as np
import pytest

import oracle_lib as O
from llmtokenizer_amd import api
from llmtokenizer_amd._lib import BpeError

pytestmark = pytest.mark.gpu

DATA = b"a" * 5000 + b"xyz" * 10
# (a, a) -> 256, (256, 256) -> 257, ...: tokens of 2, 4, ..., 4096 bytes
MERGES = np.array([[97, 97]] + [[256 + i, 256 + i] for i in range(11)], dtype=np.uint32)


def _with_end_max(v, fn):
    os.environ["BPE_END_MAX"] = str(v)
    try:
        return fn()
    finally:
        del os.environ["BPE_END_MAX"]


def test_long_run_within_limit_matches_oracle():
    assert (api.encode(DATA, MERGES) == O.encode(DATA, MERGES)).all()
    m, ids = api.train_bytes(DATA, 40)
    om, oi, _ = O.train(DATA, 40, O.EMU)
    assert (m == om).all() and (ids == oi).all()


def test_encode_stops_at_end_max():
    with pytest.raises(BpeError):
        _with_end_max(100, lambda: api.encode(DATA, MERGES))
    # a limit above the longest token: identical ids
    assert (_with_end_max(5000, lambda: api.encode(DATA, MERGES)) == O.encode(DATA, MERGES)).all()


@pytest.mark.parametrize("batch", ["1", "0"])
def test_train_stops_at_end_max(batch):
    def run():
        os.environ["BPE_BATCH"] = batch
        try:
            e = api.Engine(0)
            e.load(DATA)
            try:
                e.train(-1, fast=True)
            finally:
                e.close()
        finally:
            del os.environ["BPE_BATCH"]
    with pytest.raises(BpeError, match="out of range"):
        _with_end_max(100, run)
