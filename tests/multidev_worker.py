"""Child process of tests/test_gpu_multidev.py: one in-process multi-device
training job (bpe_train_bytes_devices) checked against the single-GPU engine
and the oracle.  Runs in its own process so that the ranks' streams and
buffers never share a process with the rest of the GPU suite.

usage: multidev_worker.py SEED NBYTES MERGES DEV[,DEV...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    seed, n, merges = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    devs = [int(x) for x in sys.argv[4].split(",")]
    from llmtokenizer_amd import api
    from llmtokenizer_amd.synth import synth_bytes
    import oracle_lib as O
    data = synth_bytes(seed, n)
    mk, idsk = api.train_bytes_devices(data, devs, merges)
    om, oids, _ = O.train(data, merges, O.RULE if n >= (1 << 20) else O.EMU)
    ok = mk.shape == om.shape and bool((mk == om).all()) and idsk.size == oids.size and bool((idsk == oids).all())
    print(f"ranks {len(devs)} merges {mk.shape[0]} ids {idsk.size} oracle-equal {ok}", flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
