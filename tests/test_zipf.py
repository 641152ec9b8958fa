"""Zipf(s = 1.1) flow mix of the synthetic generator (SURVEY.md §8(d) config 3,
"second run"): the CDF table, the host generator's flow frequencies, and the
records of such a trace through the oracle. CPU only; the device generator and
the HIP parse of the same trace are checked in test_gpu_parity.py."""
import numpy as np

import tcbee_amd
from tcbee_amd import trace


def test_zipf_cdf_table():
    nf = 10_000
    z = trace.zipf_cdf(nf)
    assert z.dtype == np.uint64 and len(z) == nf
    assert int(z[-1]) == 2 ** 64 - 1
    assert np.all(np.diff(z) > 0)  # every flow has a non-empty interval
    h = float(np.sum(np.arange(1, nf + 1, dtype=np.float64) ** -trace.ZIPF_S))
    assert abs(float(z[0]) / 2.0 ** 64 - 1.0 / h) < 1e-9
    assert len(trace.zipf_cdf(1)) == 1 and int(trace.zipf_cdf(1)[0]) == 2 ** 64 - 1


def test_zipf_host_generator_frequencies(oracle):
    n, nf = 200_000, 1000
    tr = tcbee_amd.synth_trace(n, sizes="imix", kind=trace.GEN_ZIPF, n_flows=nf)
    rec, fh, fi, ctr, table = oracle.parse(tr)
    assert len(rec) == n and ctr["handled"] == n
    assert int(table["pkts"].sum()) == n
    assert int(table["bytes"].sum()) == int(tr.caplen.sum())
    pk = np.sort(table["pkts"].astype(np.int64))[::-1]
    p = np.arange(1, nf + 1, dtype=np.float64) ** -trace.ZIPF_S
    p /= p.sum()
    # the heaviest flows carry their Zipf share (binomial counts, 5 sigma)
    for k in range(5):
        assert abs(pk[k] - n * p[k]) < 5 * np.sqrt(n * p[k]) + 1, (k, pk[k], n * p[k])
    # heavy head: far from the uniform mix of kind 1 at the same flow count
    uni = oracle.parse(tcbee_amd.synth_trace(n, sizes="imix", kind=trace.GEN_MULTI,
                                             n_flows=nf))[4]
    assert int(pk[0]) > 20 * int(uni["pkts"].max())


def test_zipf_generator_is_deterministic_and_sliceable():
    a = tcbee_amd.synth_trace(5000, sizes="64", kind=trace.GEN_ZIPF, n_flows=300)
    b = tcbee_amd.synth_trace(3000, sizes="64", kind=trace.GEN_ZIPF, n_flows=300,
                              first_index=2000)
    assert np.array_equal(a.arena[2000 * 64:], b.arena)
    c = tcbee_amd.synth_trace(5000, sizes="64", kind=trace.GEN_ZIPF, n_flows=300)
    assert np.array_equal(a.arena, c.arena)
