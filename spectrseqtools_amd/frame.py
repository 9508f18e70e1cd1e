"""A minimal column frame standing in for the polars DataFrames the hot path
and its callers read (EXPLANATION_MASSES, the nucleotide_df handed to
DynamicProgrammingTable, the fragment frames of classify_fragments /
Predictor / SkeletonBuilder).  Only the access patterns those callers use are
provided.  Any object with `columns` and `get_column(name).to_list()` -- e.g.
a real polars DataFrame -- is accepted wherever a Frame is read
(`as_columns`).
"""
import numpy as np


class Column(list):
    def to_list(self):
        return list(self)

    def min(self):
        return min(self)

    def max(self):
        return max(self)


class Frame:
    def __init__(self, columns):
        self._cols = {k: list(v) for k, v in columns.items()}
        lens = {len(v) for v in self._cols.values()}
        if len(lens) > 1:
            raise ValueError("ragged frame")

    @property
    def columns(self):
        return list(self._cols)

    def __len__(self):
        return len(next(iter(self._cols.values()), []))

    def get_column(self, name):
        return Column(self._cols[name])

    def __getitem__(self, key):
        if isinstance(key, tuple):  # frame[row, "col"] (polars item access)
            return self._cols[key[1]][key[0]]
        return self.get_column(key)

    def __setitem__(self, key, value):  # frame[row, "col"] = value (skeleton_building.py:185-186)
        row, name = key
        self._cols[name][row] = value

    def item(self, row, name):
        return self._cols[name][row]

    def get_column_index(self, name):
        return self.columns.index(name)

    def rows(self):
        return list(zip(*self._cols.values()))

    iter_rows = rows

    def filter_rows(self, predicate):
        keep = [i for i, r in enumerate(self.rows()) if predicate(dict(zip(self.columns, r)))]
        return self.take(keep)

    def filter_mask(self, mask):
        """Rows where the boolean mask is true (order kept)."""
        return self.take(np.flatnonzero(np.asarray(mask, dtype=bool)))

    def take(self, indices):
        idx = [int(i) for i in indices]
        return Frame({k: [v[i] for i in idx] for k, v in self._cols.items()})

    def sort(self, name):
        """Stable ascending sort by one column (polars sort ties: any order)."""
        order = sorted(range(len(self)), key=lambda i: self._cols[name][i])
        return self.take(order)

    def with_column(self, name, values):
        cols = dict(self._cols)
        cols[name] = list(values)
        return Frame(cols)

    def with_columns(self, **columns):
        cols = dict(self._cols)
        for k, v in columns.items():
            cols[k] = list(v)
        return Frame(cols)

    def with_row_index(self, name="index"):
        """polars with_row_index: a 0.. column put first."""
        return Frame({name: list(range(len(self))), **self._cols})

    def with_modification_rates(self, rate_of):
        """New frame whose modification_rate column is rate_of(row_dict) -- the
        cli's singleton / canonical-base rate edits (cli.py:115-139)."""
        rates = [rate_of(dict(zip(self.columns, r))) for r in self.rows()]
        return self.with_column("modification_rate", rates)

    def to_dict(self):
        return {k: list(v) for k, v in self._cols.items()}

    def write_csv(self, path, separator=","):
        with open(path, "w") as f:
            f.write(separator.join(self.columns) + "\n")
            for r in self.rows():
                f.write(separator.join("" if x is None else str(x) for x in r) + "\n")

    def __repr__(self):
        return f"Frame({len(self)} rows: {', '.join(self.columns)})"


def as_columns(frame):
    """Ordered {name: list} of a Frame, a polars / pandas DataFrame or a dict."""
    if isinstance(frame, Frame):
        return frame.to_dict()
    if isinstance(frame, dict):
        return {k: list(v) for k, v in frame.items()}
    cols = list(frame.columns)
    if hasattr(frame, "get_column"):
        return {c: list(frame.get_column(c).to_list()) for c in cols}
    return {c: list(frame[c].tolist()) for c in cols}  # pandas


def like(template, columns):
    """A frame of the same kind as `template` (polars, pandas or Frame)."""
    mod = type(template).__module__.split(".")[0]
    if mod == "polars":
        import polars as pl

        return pl.DataFrame(columns)
    if mod == "pandas":
        import pandas as pd

        return pd.DataFrame(columns)
    return Frame(columns)
