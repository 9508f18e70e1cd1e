"""A6: the .npy table cache (load_dp_table / set_table_path,
mass_table.py:142-151, :319-340) on the GPU engine: the file it writes is
byte-identical to the reference's own cache file, a cached file is read back
instead of rebuilt, and DynamicProgrammingTable(use_cache=True) -- the
reference's constructor path, through the engine's validated upload --
answers exactly as the GPU-built table does."""
import hashlib
import os

import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu

# SHA-256 of the reference's ~/.cache/spectrseqtools/dp_table/1.3/tol_1E-03.32_per_cell.npy
# (written by the reference's own load_dp_table)
REFERENCE_NPY_SHA = "5a36565b09d11c288204aad0157eaa95240f1696d1275871a4e4ef320affd6e2"


def _sha_file(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 24), b""):
            h.update(chunk)
    return h.hexdigest()


def test_load_dp_table_writes_the_reference_file(tmp_path):
    from spectrseqtools_amd import _native
    from spectrseqtools_amd.mass_table import load_dp_table

    g = load_golden("tables.json")["packed"][0]
    path = str(tmp_path / "tol_1E-03.32_per_cell")
    words = load_dp_table(path, g["masses"], engine=_native.get_engine(0))
    assert hashlib.sha256(np.ascontiguousarray(words).tobytes()).hexdigest() == g["sha256"]
    assert _sha_file(path + ".npy") == REFERENCE_NPY_SHA
    mtime = os.path.getmtime(path + ".npy")
    again = load_dp_table(path, g["masses"], engine=_native.get_engine(0))  # read, not rebuilt
    assert os.path.getmtime(path + ".npy") == mtime and np.array_equal(again, words)


def test_cached_table_answers_like_the_built_one(tmp_path, monkeypatch):
    from spectrseqtools_amd import _native, mass_table
    from spectrseqtools_amd.mass_explanation import explain_masses, is_valid_masses
    from spectrseqtools_amd.masses import EXPLANATION_MASSES, MATCHING_THRESHOLD, TOLERANCE

    monkeypatch.setattr(mass_table, "TABLE_DIR", str(tmp_path))
    seq = mass_table.SequenceInformation(max_len=6, su_mass=2000.0, obs_mass=2000.0, modification_rate=0.5)
    eng = _native.get_engine(0)
    built = mass_table.DynamicProgrammingTable(EXPLANATION_MASSES, 32, MATCHING_THRESHOLD, TOLERANCE, seq, engine=eng)
    cached = mass_table.DynamicProgrammingTable(EXPLANATION_MASSES, 32, MATCHING_THRESHOLD, TOLERANCE, seq, engine=eng,
                                                use_cache=True)
    assert os.path.exists(os.path.join(str(tmp_path), "tol_1E-03.32_per_cell.npy"))
    assert np.array_equal(cached.table, built.table)
    rng = np.random.default_rng(3)
    ms = [m.mass for m in built.masses]
    masses = np.array([sum(rng.choice(ms[1:], rng.integers(1, 4))) * 1e-3 for _ in range(400)])
    masses += rng.normal(0, 0.003, len(masses))
    assert np.array_equal(is_valid_masses(masses, cached), is_valid_masses(masses, built))
    # the uploaded table has no pair list: every window runs the general path
    a = explain_masses(masses, cached, max_modifications=3)
    b = explain_masses(masses, built, max_modifications=3)
    assert [x.explanations for x in a] == [x.explanations for x in b]
