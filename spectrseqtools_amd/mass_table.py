"""DP table objects, device-resident.

Mirror of spectrseqtools/mass_table.py (reference v0.1.2).  The packed 2-bit
unbounded-knapsack table (set_up_bit_table, :207-248) is built on the GPU by
libsstgpu.so and stays in HBM together with the engine's per-mass index; the
numpy `table` attribute is materialised only when read.
"""
import os
import pathlib
from dataclasses import dataclass
from typing import List

import numpy as np

from . import _native
from .masses import EXPLANATION_MASSES, UNMODIFIED_BASES

try:  # the reference's cache location (mass_table.py:14-16)
    from platformdirs import user_cache_dir

    TABLE_DIR = user_cache_dir(appname="spectrseqtools/dp_table", version="1.3", ensure_exists=True)
except Exception:  # pragma: no cover - platformdirs missing or home not writable
    TABLE_DIR = os.path.join(os.path.expanduser("~"), ".cache", "spectrseqtools", "dp_table", "1.3")

MAX_SEQ_LENGTH = 35  # mass_table.py:18

_DTYPES = {4: np.uint8, 8: np.uint16, 16: np.uint32, 32: np.uint64}


@dataclass
class SequenceInformation:
    max_len: int
    su_mass: float
    obs_mass: float
    modification_rate: float


@dataclass
class NucleotideMass:
    mass: int
    names: List[str]
    is_modification: bool
    modification_rate: float

    def __eq__(self, other):
        return self.mass == other.mass

    def __le__(self, other):
        return self.mass <= other.mass

    def __lt__(self, other):
        return self.mass < other.mass

    def __ge__(self, other):
        return self.mass >= other.mass

    def __gt__(self, other):
        return self.mass > other.mass


class DynamicProgrammingTable:
    """mass_table.py:52-139 with the table held on the GPU.

    Public attributes as in the reference: table (numpy, downloaded lazily),
    compression_per_cell, precision, tolerance, seq, masses.  `device_table`
    is the engine handle the query functions use.
    """

    def __init__(self, nucleotide_df, compression_rate: int, tolerance: float, precision: float,
                 seq: SequenceInformation, engine=None, use_cache=False):
        self.compression_per_cell = compression_rate
        self.tolerance = tolerance
        self.precision = precision
        self.seq = seq
        self.masses = initialize_nucleotide_masses(nucleotide_df)
        self._engine = engine
        self._device = None
        self._table_host = None

        # Adapt individual modification rates to universal one (:76-77)
        self._adapt_individual_modification_rates_by_universal_one()

        # No alphabet reduction: the full table (load_dp_table, :80-84).  By
        # default built on the GPU in milliseconds, so the table always matches
        # self.masses.  use_cache=True follows the reference exactly: read (or
        # build and write) the .npy cache at set_table_path(); the cache key
        # ignores the alphabet, and a cached table that does not follow the
        # recurrence for self.masses is rejected by the engine's upload check
        # (the reference would use it silently).
        if self._device is None:
            masses = [m.mass for m in self.masses]
            if use_cache:
                words = load_dp_table(set_table_path(precision, compression_rate), masses, engine=self._engine)
                self._set_device(_native.DeviceTable.upload(masses, words, compression_rate, engine=self._engine))
                self._table_host = words
            else:
                self._set_device(_native.DeviceTable.build(masses, max(masses) * MAX_SEQ_LENGTH, compression_rate,
                                                           engine=self._engine))

    # -- device table ---------------------------------------------------------
    def close(self):
        """Free the device table now (HBM is not Python memory: a table held
        by a reference cycle would otherwise wait for a full GC pass)."""
        self._set_device(None)

    def _set_device(self, dev):
        if self._device is not None:
            self._device.close()
        self._device = dev
        self._table_host = None

    @property
    def device_table(self):
        """Engine table with the budgets the explain DFS reads pushed to it:
        is_modification and round(seq.max_len * modification_rate) per row
        (mass_explanation.py:158-172, :200)."""
        is_mod = [m.is_modification for m in self.masses]
        caps = [round(self.seq.max_len * m.modification_rate) for m in self.masses]
        self._device.set_budgets(is_mod, caps)
        return self._device

    @property
    def table(self):
        if self._table_host is None:
            self._table_host = self._device.download()
        return self._table_host

    @table.setter
    def table(self, words):
        words = np.ascontiguousarray(words)
        c = {np.dtype(v): k for k, v in _DTYPES.items()}.get(words.dtype)
        if c is None:
            raise TypeError(f"unsupported DP table dtype {words.dtype}")
        self._set_device(_native.DeviceTable.upload([m.mass for m in self.masses], words, c, engine=self._engine))

    # -- alphabet adaptation (mass_table.py:86-121) ----------------------------
    def _adapt_individual_modification_rates_by_universal_one(self):
        for nucleotide_mass in self.masses:
            if not nucleotide_mass.is_modification:
                continue
            if nucleotide_mass.modification_rate > self.seq.modification_rate:
                nucleotide_mass.modification_rate = self.seq.modification_rate
        self._reduce_nucleotide_list()

    def adapt_individual_modification_rates_by_alphabet_reduction(self, alphabet):
        for nucleotide_mass in self.masses:
            if not nucleotide_mass.is_modification:
                continue
            if all(name not in alphabet for name in nucleotide_mass.names):
                nucleotide_mass.modification_rate = 0.0
        self._reduce_nucleotide_list()

    def _reduce_nucleotide_list(self):
        new_masses = [mass for mass in self.masses if mass.mass == 0.0 or mass.modification_rate > 0.0]
        if len(new_masses) == len(self.masses):
            return
        integer_masses = [mass.mass for mass in new_masses]
        self._set_device(_native.DeviceTable.build(integer_masses, max(integer_masses) * MAX_SEQ_LENGTH,
                                                   self.compression_per_cell, engine=self._engine))
        self.masses = new_masses

    def print_masses(self):
        """mass_table.py:123-139 (plain-text rendering of the same rows)."""
        names = set()
        for mass in self.masses:
            names.update(mass.names)
        rows = sorted((r for r in EXPLANATION_MASSES.rows() if r[1] in names), key=lambda r: r[0])
        rates = [mass.modification_rate for mass in self.masses[1:]]
        print("monoisotopic_mass\tnucleoside\tmodification_rate")
        for r, rate in zip(rows, rates):
            print(f"{r[0]}\t{r[1]}\t{rate}")

    def __repr__(self):
        return (f"DynamicProgrammingTable(rows={len(self.masses)}, compression_per_cell={self.compression_per_cell}, "
                f"precision={self.precision}, tolerance={self.tolerance}, seq={self.seq})")


def set_table_path(precision, compression_rate):
    """mass_table.py:142-151."""
    path = f"{TABLE_DIR}/tol_{precision:.0E}.{compression_rate}_per_cell"
    subdir = "/".join(path.split("/")[:-1])
    if not os.path.exists(subdir):
        os.makedirs(subdir)
    return path


def initialize_nucleotide_masses(nucleotide_df):
    """mass_table.py:154-204."""
    ints_col = nucleotide_df.get_column("tolerated_integer_masses").to_list()
    names_col = nucleotide_df.get_column("nucleoside").to_list()
    rates_col = nucleotide_df.get_column("modification_rate").to_list()
    integer_masses = sorted(set(list(ints_col) + [0]))
    names, rates = {}, {}
    for m, n, r in zip(ints_col, names_col, rates_col):
        names.setdefault(m, []).append(n)
        rates.setdefault(m, []).append(r)
    is_mod = {m: any(base not in UNMODIFIED_BASES for base in names[m]) for m in names}
    return [
        NucleotideMass(mass, names[mass], is_mod[mass], max(rates[mass])) if mass != 0
        else NucleotideMass(0, [], False, 0.0)
        for mass in integer_masses
    ]


def set_up_bit_table(integer_masses, max_mass: int, compression_rate: int, engine=None):
    """mass_table.py:207-248, computed by the GPU engine; returns the packed
    ndarray (bit-identical to the reference's)."""
    select_table_building_settings(compression_rate)
    dev = _native.DeviceTable.build(list(integer_masses), int(max_mass), compression_rate, engine=engine)
    try:
        return dev.download()
    finally:
        dev.close()


def select_table_building_settings(compression_rate: int):
    """mass_table.py:251-289."""
    match compression_rate:
        case 4:
            return {"type": np.uint8, "init": 0xC0, "alt_first": 0xAA, "alt_sec": 0x55, "full": np.uint8(0xFF)}
        case 8:
            return {"type": np.uint16, "init": 0xC000, "alt_first": 0xAAAA, "alt_sec": 0x5555,
                    "full": np.uint16(0xFFFF)}
        case 16:
            return {"type": np.uint32, "init": 0xC0000000, "alt_first": 0xAAAAAAAA, "alt_sec": 0x55555555,
                    "full": np.uint32(0xFFFFFFFF)}
        case 32:
            return {"type": np.uint64, "init": 0xC000000000000000, "alt_first": 0xAAAAAAAAAAAAAAAA,
                    "alt_sec": 0x5555555555555555, "full": np.uint64(0xFFFFFFFFFFFFFFFF)}
        case _:
            raise ValueError(f"The compression rate {compression_rate} is not compatible with the table setup.")


def load_dp_table(table_path, integer_masses, engine=None):
    """mass_table.py:319-340: read the .npy cache or build (on the GPU) and save it."""
    compression_rate = int(table_path.split(".")[-1].rstrip("_per_cell"))
    max_mass = max(integer_masses) * MAX_SEQ_LENGTH
    if not pathlib.Path(f"{table_path}.npy").is_file():
        print("Table not found")
        if compression_rate == 1:
            raise NotImplementedError("compression 1 (set_up_mass_table) is not provided by the GPU engine")
        dp_table = set_up_bit_table(integer_masses, max_mass, compression_rate, engine=engine)
        np.save(table_path, dp_table)
    return np.load(f"{table_path}.npy", allow_pickle=False)


def compute_sequence_length_bound(dp_table: DynamicProgrammingTable, dir: str) -> int:
    """Return bound on length for any sequence that could explain the given mass
    (mass_table.py:343-487), on the GPU: the reference's memoised backtrack --
    same first-visit budgets, same defaults and quirks -- see DESIGN.md."""
    if dir not in ("lower", "upper"):
        raise NotImplementedError(f"Support for '{dir}' is currently not given.")
    seq = dp_table.seq
    out = compute_sequence_length_bounds(dp_table, [seq.su_mass], [seq.obs_mass], dir)
    return int(out[0])


def compute_sequence_length_bounds(dp_table: DynamicProgrammingTable, su_masses, obs_masses, dir: str):
    """Batched compute_sequence_length_bound over (su_mass, obs_mass) pairs that
    share dp_table.seq's max_len / modification_rate (one launch)."""
    if dir not in ("lower", "upper"):
        raise NotImplementedError(f"Support for '{dir}' is currently not given.")
    seq = dp_table.seq
    max_mods = round(seq.modification_rate * seq.max_len)  # mass_table.py:351
    vals, st = dp_table.device_table.length_bound(su_masses, obs_masses, dp_table.tolerance, dp_table.precision,
                                                  seq.max_len, max_mods, dir)
    bad = np.flatnonzero(st != 0)
    if len(bad):
        s = int(st[bad[0]])
        if s == _native.SST_OUT_OF_TABLE:
            # the reference formats its window-loop variable `value` (mass_table.py:383-387, :461): the first
            # window value at or beyond the table end (the DFS only moves to smaller masses)
            k = bad[0]
            target = int(round(float(su_masses[k]) / dp_table.precision, 0))
            thr = int(np.ceil(dp_table.tolerance * float(obs_masses[k]) / dp_table.precision))
            value = max(target - thr, dp_table.device_table.n_cols * dp_table.compression_per_cell)
            raise NotImplementedError(f"The value {value} is not in the DP table. Extend its size if you want to "
                                      f"compute larger masses.")
        if s == _native.SST_LB_EMPTY_WINDOW:
            raise ValueError("min() arg is an empty sequence")
        raise RuntimeError(f"length bound aborted: DFS node budget exhausted (status {s})")
    return vals
