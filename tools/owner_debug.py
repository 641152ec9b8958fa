"""Debug helper: run the owner exchange GPU worker and report id mismatches."""
import os
import socket
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch.multiprocessing as mp

    import dist_worker
    from oracle_py import Oracle
    from tracegen import mixed_trace
    world, n, flows, cap = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    d = tempfile.mkdtemp()
    mp.spawn(dist_worker.run_gpu, args=(world, port, n, cap, d, "owner", flows, 0),
             nprocs=world, join=True)
    tr = mixed_trace(n, seed=404, n_flows=flows)
    rec, fh, fi, ctr, table = Oracle().parse(tr)
    res = [np.load(os.path.join(d, f"rank{r}.npz")) for r in range(world)]
    off = 0
    for r, x in enumerate(res):
        g = x["gids"]
        want = fi[off:off + len(g)]
        bad = np.nonzero(g != want)[0]
        print("rank", r, "records", len(g), "bad", len(bad), "status", x["status"], flush=True)
        if len(bad):
            b = bad[:10]
            print("  got", g[b], "want", want[b], "owner(want)", (fh[off + b] % world), flush=True)
            wrong_flows = np.unique(want[bad])
            print("  distinct wrong flows", len(wrong_flows), "of", len(np.unique(want)),
                  "owners", np.bincount(fh[off + bad] % world, minlength=world), flush=True)
        off += len(g)


if __name__ == "__main__":
    main()
