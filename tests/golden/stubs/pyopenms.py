"""Stand-in for pyopenms (OpenMS C++ bindings, absent offline and not even in the
reference's requirements.txt), used ONLY by tests/golden/make_golden.py so that
the reference's own medoid driver ``most_similar_representative.main`` runs for
real: its cluster scan, distance-matrix fill, pandas pairwise sums, argmin and
tie-breaking are the reference's code; only the three OpenMS entry points it
calls are restated here.

* ``XQuestScores.xCorrelationPrescore(s1, s2, tol)`` -- restated from OpenMS
  ``XQuestScores.cpp`` (version unpinned): empty -> 0; table size
  ``ceil(max(last mz)/tol)+1``; binary tables set at ``(size_t)ceil(mz/tol)``;
  f64 dot product; divided by ``min(#peaks)``.  SURVEY.md Appendix A.3.
  PARITY UNPINNED at this boundary: no OpenMS test vector exists offline.
* ``MascotGenericFile.load/store`` -- minimal MGF reader/writer: every
  ``mz intensity`` line is a peak (no sorting, no zero-intensity removal; the
  synthetic fixtures are sorted with intensities > 0, where both choices agree).
  ``store`` writes the chosen spectra's titles, one per line, which is all the
  golden capture needs.
"""
import math

import numpy as np

__all__ = ["MSExperiment", "MSSpectrum", "MascotGenericFile", "XQuestScores"]


class _Peak:
    __slots__ = ("mz", "intensity")

    def __init__(self, mz, intensity):
        self.mz = mz
        self.intensity = intensity

    def getMZ(self):
        return self.mz

    def getIntensity(self):
        return self.intensity


class MSSpectrum:
    def __init__(self):
        self._peaks = []
        self._meta = {}
        self.index = -1  # position in the loaded file (golden capture only)

    def size(self):
        return len(self._peaks)

    def empty(self):
        return not self._peaks

    def __len__(self):
        return len(self._peaks)

    def __getitem__(self, i):
        return self._peaks[i]

    def push_back(self, peak):
        self._peaks.append(peak)

    def setMetaValue(self, key, value):
        self._meta[key] = value.encode() if isinstance(value, str) else value

    def getMetaValue(self, key):
        return self._meta[key]

    def mz_array(self):
        return np.fromiter((p.mz for p in self._peaks), np.float64, len(self._peaks))


class MSExperiment:
    def __init__(self):
        self._spectra = []

    def size(self):
        return len(self._spectra)

    def __getitem__(self, i):
        return self._spectra[i]

    def addSpectrum(self, spec):
        self._spectra.append(spec)


class MascotGenericFile:
    def load(self, path, exp):
        cur = None
        with open(path) as fh:
            for raw in fh:
                line = raw.strip()
                if line == "BEGIN IONS":
                    cur = MSSpectrum()
                elif line == "END IONS":
                    cur.index = exp.size()
                    exp.addSpectrum(cur)
                    cur = None
                elif cur is None or not line:
                    continue
                elif "=" in line and not line[0].isdigit():
                    k, v = line.split("=", 1)
                    cur.setMetaValue(k, v)
                else:
                    mz, inten = line.split()[:2]
                    cur.push_back(_Peak(float(mz), float(inten)))

    def store(self, path, exp):
        with open(path, "w") as fh:
            for i in range(exp.size()):
                s = exp[i]
                fh.write(f"{s.index}\t{s.getMetaValue('TITLE').decode()}\n")


class XQuestScores:
    def xCorrelationPrescore(self, spec1, spec2, tolerance):
        if spec1.empty() or spec2.empty():
            return 0.0
        max_ion = max(spec1[spec1.size() - 1].getMZ(), spec2[spec2.size() - 1].getMZ())
        table_size = int(math.ceil(max_ion / tolerance)) + 1
        t1 = np.zeros(table_size)
        t2 = np.zeros(table_size)
        t1[np.ceil(spec1.mz_array() / tolerance).astype(np.int64)] = 1.0
        t2[np.ceil(spec2.mz_array() / tolerance).astype(np.int64)] = 1.0
        dot = 0.0
        for v in (t1 * t2)[(t1 * t2) != 0]:  # sequential f64 sum; values are 0/1 so exact
            dot += v
        peaks = float(min(spec1.size(), spec2.size()))
        return dot / peaks
