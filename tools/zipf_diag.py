"""Diagnose a Zipf many-flow mismatch (tests/test_gpu_parity.py::test_zipf_many_flows):
runs the case on the library TCBEE_AB_LIB selects and prints which flows differ from
the oracle (first_seen / pkts / bytes) and how many record ids differ."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    import tcbee_amd
    from oracle_py import Oracle
    oracle = Oracle()
    flows = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    n = 4_000_000
    tr = tcbee_amd.synth_trace(n, sizes="imix", kind=2, n_flows=flows, seed=flows + 2)
    ft = oracle.new_flowtab(1 << 21)
    rec, fh, fi, ctr, _ = oracle.parse(tr, ft=ft)
    if os.environ.get("ZD_SHIFT"):  # a different trace for the same context sizes
        pass
    table = oracle.flows(ft)
    oracle.free_flowtab(ft)
    d_arena = torch.from_numpy(np.concatenate([tr.arena, np.zeros(64, np.uint8)])).cuda()
    d_off = torch.from_numpy(tr.offset.view(np.int64)).cuda()
    d_len = torch.from_numpy(tr.caplen.view(np.int32)).cuda()
    d_ts = torch.from_numpy(tr.ts_ns.view(np.int64)).cuda()
    rec_d = torch.empty(n * 74 + 64, dtype=torch.uint8, device="cuda")
    fi_d = torch.empty(n, dtype=torch.int32, device="cuda")
    n_d = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctr_d = torch.zeros(4, dtype=torch.int64, device="cuda")
    fresh = os.environ.get("ZD_FRESH") == "1"  # a new context per rep, as the test does
    p = tcbee_amd.PacketParser(max_frames=n, max_flows=flows + flows // 16)
    if True:
        for r in range(reps):
            if fresh and r:
                p.close()
                p = tcbee_amd.PacketParser(max_frames=n, max_flows=flows + flows // 16)
            elif not fresh:
                p.reset_flows()
            ctr_d.zero_()
            fi_d.fill_(-2)  # a sentinel: an id K3 never wrote shows as a mismatch
            rec_d.fill_(0x5A)
            s = torch.cuda.current_stream().cuda_stream
            p.parse_device(d_arena, len(tr.arena), d_off, d_len, d_ts, n, rec_d, n, None, fi_d,
                           n_d, ctr_d, stream=s)
            torch.cuda.synchronize()
            g = p.flows()
            gi = fi_d.cpu().numpy().view(np.uint32)
            bad_ids = int((gi != fi).sum())
            unwritten = int((gi == 0xFFFFFFFE).sum())
            rbad = int(np.any(rec_d[:n * 74].cpu().numpy().reshape(-1, 74) != rec, axis=1).sum())
            msg = f"rep {r}: flows gpu {len(g)} oracle {len(table)}, ids differ {bad_ids} (unwritten {unwritten}, records differ {rbad}), mode {p.count_mode()}, status {p.status()}"
            if len(g) == len(table):
                for k in ("tuple", "pkts", "bytes", "first_seen"):
                    d = np.nonzero(np.any((g[k] != table[k]).reshape(len(g), -1), axis=1))[0]
                    msg += f"; {k} differ {len(d)}" + (f" first {d[:3].tolist()}" if len(d) else "")
                if len(np.nonzero(g["first_seen"] != table["first_seen"])[0]):
                    d = np.nonzero(g["first_seen"] != table["first_seen"])[0][:3]
                    msg += f"; fs gpu {g['first_seen'][d].tolist()} oracle {table['first_seen'][d].tolist()}"
            print(msg, flush=True)
    p.close()


if __name__ == "__main__":
    main()
