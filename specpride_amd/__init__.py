"""specpride_amd -- MI355X-native consensus/representative-spectrum engine.

Drop-in for the hot path of timosachsenberg/specpride (cluster -> consensus or
representative spectrum): bin-mean (``binning.py``), gap-average
(``average_spectrum_clustering.py``) and medoid
(``most_similar_representative.py``).  Host code packs clusters into a
cluster-segmented CSR batch (:mod:`specpride_amd.csr`) and hands it to
hand-written gfx950 HIP kernels through the C-ABI in ``include/specpride.h``
(:mod:`specpride_amd.engine`).  See DESIGN.md.
"""
__version__ = "0.1.0"
