"""Debug: 1M-flow device parse vs the oracle, mismatch anatomy (round 3)."""
import os, sys
# TCBEE_* variants / ablations are dispatched by the variants build only
os.environ.setdefault("TCBEE_AB_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tcbee_amd", "lib", "libtcbee_amd_variants.so"))
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import torch
import tcbee_amd
from oracle_py import Oracle

def run(cap_mult, n=3_500_000, flows=1_000_000, env=None):
    for k, v in (env or {}).items():
        os.environ[k] = v
    tr = tcbee_amd.synth_trace(n, sizes="imix", kind=1, n_flows=flows)
    d_arena = torch.from_numpy(np.concatenate([tr.arena, np.zeros(64, np.uint8)])).cuda()
    d_off = torch.from_numpy(tr.offset.view(np.int64)).cuda()
    d_len = torch.from_numpy(tr.caplen.view(np.int32)).cuda()
    d_ts = torch.from_numpy(tr.ts_ns.view(np.int64)).cuda()
    rec_d = torch.empty(n * 74 + 64, dtype=torch.uint8, device="cuda")
    fh_d = torch.empty(n, dtype=torch.int32, device="cuda")
    fi_d = torch.empty(n, dtype=torch.int32, device="cuda")
    n_d = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctr_d = torch.zeros(4, dtype=torch.int64, device="cuda")
    orc = Oracle()
    ft = orc.new_flowtab(1 << 21)
    rec, fh, fi, ctr, _ = orc.parse(tr, ft=ft)
    table = orc.flows(ft)
    orc.free_flowtab(ft)
    for rep in range(2):
        with tcbee_amd.PacketParser(max_frames=n, max_flows=cap_mult * flows) as p:
            s = torch.cuda.current_stream().cuda_stream
            p.parse_device(d_arena, len(tr.arena), d_off, d_len, d_ts, n, rec_d, n, fh_d, fi_d, n_d,
                           ctr_d, stream=s)
            torch.cuda.synchronize()
            gi = fi_d.cpu().numpy().view(np.uint32)
            fl = p.flows()
            bad = np.nonzero(gi != fi)[0]
            tab_ok = len(fl) == len(table) and np.array_equal(fl, table)
            fs_bad = np.nonzero(fl["first_seen"] != table["first_seen"])[0] if len(fl) == len(table) else []
            pk_bad = np.nonzero(fl["pkts"] != table["pkts"])[0] if len(fl) == len(table) else []
            print(f"cap{cap_mult} rep{rep} env={env}: flows {len(fl)}/{len(table)} table_ok={tab_ok} "
                  f"bad_ids={len(bad)} first={bad[:5].tolist()} chunks={np.unique(bad // 12288)[:10].tolist()} "
                  f"fs_bad={len(fs_bad)} pk_bad={len(pk_bad)} status={p.status()} mode={p.count_mode()}",
                  flush=True)
            if len(bad):
                print("  gpu ids", gi[bad[:5]].tolist(), "oracle", fi[bad[:5]].tolist(), flush=True)

torch.cuda.set_device(0)
torch.cuda.set_stream(torch.cuda.Stream())
run(1)
run(1, env={"TCBEE_K3ABL": "91"})
run(1, env={"TCBEE_K3ABL": "93"})
run(4, env={"TCBEE_K3ABL": "0"})
