"""TEST INFRASTRUCTURE: a CPU stand-in for _native.DeviceTable backed by the
oracle (oracle/sst_oracle.c), so that the host-side mirrors of the
reference's callers (classify_fragments, Predictor, SkeletonBuilder) run in
the CPU suite.  Installed only by tests (monkeypatch of DeviceTable.build);
the product path has no CPU fallback (tests/test_boundary.py)."""
import numpy as np

import _oracle as oracle
from spectrseqtools_amd import _native


class FakeResult:
    def __init__(self, status, sols):
        self.n = len(status)
        self.status = np.asarray(status, dtype=np.int8)
        self.count = np.array([len(s) for s in sols], dtype=np.uint64)
        self._sols = sols

    def candidates(self, i):
        return list(self._sols[i])


class FakeEngine:
    device = -1

    @staticmethod
    def is_singleton(integer_masses, masses, thresholds, tolerance, precision):
        return oracle.is_singleton_batch(masses, thresholds, integer_masses, tolerance, precision).astype(np.int8)


class FakeDeviceTable:
    compression = 32

    def __init__(self, masses, max_mass, compression):
        assert compression == 32
        self.masses = [int(m) for m in masses]
        self.table = oracle.build_table(self.masses, int(max_mass), compression)
        self.n_cols = self.table.shape[1]
        self.engine = FakeEngine()
        self.alph = None
        self.calls = 0

    def set_budgets(self, is_mod, caps):
        self.alph = oracle.Alphabet(self.masses, is_mod, caps)

    def close(self):
        self.table = None

    def is_valid(self, masses, thresholds, tolerance, precision):
        self.calls += 1
        return oracle.is_valid_batch(self.table, 32, masses, thresholds, tolerance, precision=precision)

    def is_valid_peaks(self, observed, shifts, tolerance, precision):
        self.calls += 1
        o = np.asarray(observed, dtype=np.float64)
        su = np.concatenate([o - s for s in shifts]) if len(shifts) else np.zeros(0)
        return oracle.is_valid_batch(self.table, 32, su, tolerance * np.tile(o, len(shifts)), tolerance,
                                     precision=precision)

    def explain(self, masses, thresholds, tolerance, precision, max_mods, with_memo=True, cap=2 ** 32):
        self.calls += 1
        masses = np.asarray(masses, dtype=np.float64)
        A = np.broadcast_to(np.asarray(max_mods, dtype=np.float64), masses.shape)
        st, sols = [], []
        for i, m in enumerate(masses):
            a = "inf" if not np.isfinite(A[i]) else int(A[i])
            t = None if thresholds is None else float(thresholds[i])
            s, rows, n_empty, _ = oracle.explain_table(self.table, 32, self.alph, float(m), t, tolerance, a,
                                                       with_memo=with_memo, precision=precision)
            if s == -1:
                st.append(_native.SST_OUT_OF_TABLE)
                sols.append([])
            elif s == 0:
                st.append(_native.SST_NONE)
                sols.append([])
            elif rows:
                st.append(_native.SST_SOME)
                sols.append(rows)
            else:
                st.append(_native.SST_EMPTY)
                sols.append([])
        return FakeResult(st, sols)


def install(monkeypatch):
    """Route DynamicProgrammingTable's device tables to the oracle."""
    monkeypatch.setattr(_native.DeviceTable, "build",
                        classmethod(lambda cls, masses, max_mass, compression, engine=None:
                                    FakeDeviceTable(masses, max_mass, compression)))
