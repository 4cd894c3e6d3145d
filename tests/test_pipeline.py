"""Tier-2 host pipeline (specpride_amd.pipeline): chunk planning on CPU, and on the GPU
the chunked, overlapped bin-mean + medoid equal to the one-batch engine call and the
C oracle (bit-exact) whatever the chunk size.  Reference: binning.py:286-302 (the
CLI's parse -> per-cluster cores flow), :170-231, most_similar_representative.py:60-111."""
import numpy as np
import pytest

from specpride_amd.pipeline import plan_chunks
from specpride_amd.synthetic import make_clusters_np


def test_plan_chunks_cover_clusters_in_order():
    csr = make_clusters_np(300, seed=5)
    so, co = csr.spec_off, csr.cluster_off
    for chunk_bytes in (1, 16 * 1000, 16 * 50_000, 1 << 40):
        chunks = plan_chunks(co, so, chunk_bytes)
        assert chunks[0][0] == 0 and chunks[-1][1] == csr.n_clusters
        assert all(a < b for a, b in chunks)
        assert all(chunks[i][1] == chunks[i + 1][0] for i in range(len(chunks) - 1))
        per = max(1, chunk_bytes // 16)
        for a, b in chunks:  # within budget, or a single cluster
            assert b - a == 1 or so[co[b]] - so[co[a]] <= per
    assert plan_chunks(np.zeros(1, np.int64), np.zeros(1, np.int64), 1 << 20) == []


@pytest.mark.gpu
@pytest.mark.parametrize("chunk_bytes", [16 * 20_000, 16 * 300_000, 1 << 34])
def test_pipeline_equals_engine_and_oracle(gpu, chunk_bytes):
    from oracle import c_oracle
    from specpride_amd import engine
    from specpride_amd.pipeline import HostPipeline

    sizes = np.concatenate([np.random.default_rng(3).integers(1, 51, 700), [70, 130]])  # + large-path medoids
    csr = make_clusters_np(len(sizes), seed=21, sizes=sizes)
    pipe = HostPipeline(chunk_bytes=chunk_bytes)
    for _ in range(2):  # the second call reuses the slots
        r = pipe.run(csr)
        assert pipe.timing["chunks"] >= (2 if chunk_bytes < 16 * csr.n_peaks else 1)
        ref = c_oracle.bin_mean(csr)
        for k in ("status", "out_off", "out_mz", "out_int", "prec", "charge"):
            np.testing.assert_array_equal(r[k], ref[k], err_msg=k)
        np.testing.assert_array_equal(r["rep"], c_oracle.medoid(csr))
    one = engine.bin_mean(engine.DeviceBatch.from_host(csr)).to_host()
    np.testing.assert_array_equal(r["out_mz"], one["out_mz"])


def _with_wide_overflow(csr, n_spec=40, n_peaks=700, seed=9):
    """csr + one small cluster (n <= 64, <= 32,768 peaks) whose ~16k distinct
    0.1-Da bins overflow the medoid wide kernel's 6,080: deferred at RUN time."""
    from specpride_amd.csr import SpectraCSR

    rng = np.random.default_rng(seed)
    mz = np.sort(np.round(rng.uniform(100.0, 2000.0, (n_spec, n_peaks)), 5), axis=1).ravel()
    inten = np.round(rng.uniform(1.0, 1000.0, mz.size), 2)
    so = np.concatenate([csr.spec_off, csr.spec_off[-1] + n_peaks * np.arange(1, n_spec + 1)])
    co = np.concatenate([csr.cluster_off, [csr.cluster_off[-1] + n_spec]])
    S = n_spec
    return SpectraCSR(co, so, np.concatenate([csr.mz, mz]), np.concatenate([csr.inten, inten]),
                      np.concatenate([csr.prec_mz, np.full(S, 500.0)]), np.concatenate([csr.charge, np.full(S, 2)]),
                      np.concatenate([csr.rt, np.zeros(S)]))


@pytest.mark.gpu
def test_pipeline_runtime_medoid_deferral_resolved_after_loop(gpu):
    """A chunk whose medoid defers a cluster at run time (large path off in that
    chunk) is re-run by the checked call after the overlapped loop; results equal
    the oracle's (no device-wide sync inside the loop)."""
    from oracle import c_oracle
    from specpride_amd.pipeline import HostPipeline

    csr = _with_wide_overflow(make_clusters_np(400, seed=31))
    pipe = HostPipeline(chunk_bytes=16 * 60_000)
    r = pipe.run(csr)
    assert pipe.timing["chunks"] >= 3 and pipe.timing["redo_chunks"] == 1
    np.testing.assert_array_equal(r["rep"], c_oracle.medoid(csr))
    ref = c_oracle.bin_mean(csr)
    for k in ("status", "out_off", "out_mz", "out_int"):
        np.testing.assert_array_equal(r[k], ref[k], err_msg=k)
