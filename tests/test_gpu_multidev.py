"""GPU parity of one training job over several devices of ONE process
(bpe_train_bytes_devices / compress with BPE_DEVICES: SURVEY 8(b)'s device
count for the C drop-in).  On the one-GPU test box every rank sits on device
0, which exercises the whole in-process protocol (direct mailbox pointers,
one host thread per rank, concurrent graph replays) except the xGMI hop.
Bar: merges and ids bit-exact with the oracle (RULE from 2^20 bytes, where
the sharded tie rule is the reference's; EMU below, where one device trains).
Every case runs in a child process (tests/multidev_worker.py): see
DESIGN.md 8 for why the ranks do not share a process with the rest of the
suite."""
import os
import subprocess
import sys

import numpy as np
import pytest

from llmtokenizer_amd.synth import synth_bytes

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _worker(*args):
    r = subprocess.run([sys.executable, os.path.join(HERE, "multidev_worker.py"), *map(str, args)],
                       capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.parametrize("ranks,merges", [(2, 300), (3, 200)])
def test_devices_equal_oracle(ranks, merges):
    _worker(5, (3 << 20) + 12345, merges, ",".join(["0"] * ranks))


def test_small_corpus_trains_on_one_device():
    # below 2^20 bytes the static-schedule emulation (one device) is used
    _worker(7, 50000, 100, "0,0")


def test_too_many_ranks_per_device_refused():
    r = subprocess.run([sys.executable, os.path.join(HERE, "multidev_worker.py"), "9", str(1 << 20), "10", "0,0,0,0"],
                       capture_output=True, text=True, timeout=150)
    assert r.returncode != 0 and "more than 3 ranks" in r.stderr


def test_compress_env_devices(tmp_path):
    # the unchanged C entry point picks the multi-device path from the environment
    data = synth_bytes(8, (1 << 20) + 999)
    path = tmp_path / "corpus.txt"
    path.write_bytes(data)
    code = ("import sys, numpy as np; sys.path.insert(0, %r); sys.path.insert(0, %r); "
            "from llmtokenizer_amd import api; import oracle_lib as O; "
            "m, ids = api.compress(%r); om, oids, _ = O.train(open(%r, 'rb').read(), 120, O.RULE); "
            "sys.exit(0 if (m.shape == om.shape and (m == om).all() and (ids == oids).all()) else 1)"
            % (ROOT, HERE, str(path), str(path)))
    env = dict(os.environ, BPE_DEVICES="0,0", BPE_MAX_MERGES="120")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stdout + r.stderr
