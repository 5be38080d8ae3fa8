"""One rank of a P2P shard group (tests/test_gpu_p2p.py starts W of them on
the same GPU): gloo carries the mailbox handles, the library does the rest.

usage: p2p_worker.py RANK WORLD PORT OUT.npz MODE DATA MERGES CUTS [MERGES.npz]
MODE: train | encode (encode: the merge list in MERGES.npz)
DATA: synth:SEED:N | alpha:SEED:N:LETTERS (tests/test_gpu_p2p.py corpus())"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    rank, world, port = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    out, mode, spec, mm = sys.argv[4], sys.argv[5], sys.argv[6], int(sys.argv[7])
    cuts = [int(x) for x in sys.argv[8].split(",")]
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    from llmtokenizer_amd import dist as bdist
    from test_gpu_p2p import corpus
    data = corpus(spec)
    mine = data[cuts[rank]:cuts[rank + 1]]
    g = bdist.p2p_group(0, mm)
    assert g.transport() == "p2p"
    g.load(0, mine)
    if mode == "train":
        g.train(mm)
        st = g.stats()
        np.savez(out, merges=g.merges(), ids=g.ids(0),
                 stats=np.array([st["ms_train"], st["spec_hits"], st["spec_misses"], st["batches"]], dtype=np.float64))
    else:
        merges = np.load(sys.argv[9])["merges"]
        g.encode(merges)
        np.savez(out, ids=g.ids(0), path=np.array([g.stats()["enc_path"]]))
    dist.barrier()
    g.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
