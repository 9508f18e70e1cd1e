"""Minimal pandas-backed stand-in for the subset of `polars` that the reference's
hot-path modules (masses.py, mass_table.py, mass_explanation.py) touch at import
time and in `DynamicProgrammingTable`, plus the frame plumbing of
fragment_classification.classify_fragments (lit, struct.map_elements, concat,
with_row_index, rename, drop, comparisons, str.contains), and of the reference's
Predictor.filter_by_explanation and SkeletonBuilder._predict_skeleton
(DataFrame.item, row/column assignment) and build_skeleton's fragment
bookkeeping (clone, vstack, when/then/otherwise, reverse subtraction).

TEST INFRASTRUCTURE ONLY.  polars is not installed in this image and there is no
network.  This module is put on sys.path solely by tests/golden/make_golden.py
(which runs in the build container, never on the GPU box) so that the
reference's own Python can be executed unmodified to produce golden vectors.
It implements frame plumbing only (CSV read, column round/add/div, group-by with
first/unique/max, left join, filter, sort); every number on the hot path is
computed by the reference's own numpy/Python code.  The alphabet it yields is
cross-checked in make_golden.py against an independent numpy restatement.
"""
import numpy as np
import pandas as pd

Int64 = "Int64"
Float64 = "Float64"
String = "String"
Boolean = "Boolean"
UInt32 = "UInt32"


class Expr:
    def __init__(self, fn, name, agg="first"):
        self.fn = fn
        self.name = name
        self.agg = agg

    def _map(self, g, name=None):
        return Expr(lambda df: g(self.fn(df)), name or self.name, self.agg)

    # arithmetic ---------------------------------------------------------
    def round(self, decimals=0):
        return self._map(lambda x: np.round(x.astype(float), decimals))

    def add(self, v):
        return self._map(lambda x: x + v)

    __add__ = add

    def __sub__(self, v):
        return self._map(lambda x: x - v)

    def __rsub__(self, v):  # int - Expr (build_skeleton's reverse end indices)
        return self._map(lambda x: v - x)

    def __truediv__(self, v):
        return self._map(lambda x: x / v)

    def __eq__(self, v):  # noqa: D105 - expression equality, not identity
        return self._map(lambda x: x == v)

    def __gt__(self, v):
        return self._map(lambda x: x > v)

    def __lt__(self, v):
        return self._map(lambda x: x < v)

    def __ge__(self, v):
        return self._map(lambda x: x >= v)

    def __le__(self, v):
        return self._map(lambda x: x <= v)

    def __and__(self, o):
        return Expr(lambda df: self.fn(df) & o.fn(df), self.name)

    def __or__(self, o):
        return Expr(lambda df: self.fn(df) | o.fn(df), self.name)

    def __invert__(self):
        return self._map(lambda x: ~x)

    @property
    def str(self):
        outer = self

        class _Str:
            def contains(self, pat):
                return outer._map(lambda x: x.astype(str).str.contains(pat, regex=True))

        return _Str()

    def map_elements(self, fn, return_dtype=None):
        return self._map(lambda rows: pd.Series([fn(r) for r in rows]))

    __hash__ = object.__hash__

    def alias(self, name):
        return Expr(self.fn, name, self.agg)

    def cast(self, dtype):
        return self._map(lambda x: x.astype("int64") if dtype == Int64 else x)

    def is_in(self, values):
        vals = list(values)
        return self._map(lambda x: x.isin(vals))

    # aggregations (only meaningful inside group_by().agg) ----------------
    def first(self):
        return Expr(self.fn, self.name, "first")

    def unique(self):
        return Expr(self.fn, self.name, "unique")

    def max(self):
        return Expr(self.fn, self.name, "max")


def col(name):
    return Expr(lambda df: df._d[name], name)


def lit(value, dtype=None):
    return Expr(lambda df: pd.Series([value] * len(df._d)), "literal")


def struct(*names):
    return Expr(lambda df: [dict(zip(names, r)) for r in df._d[list(names)].itertuples(index=False)], names[0])


def _values(e, df):
    return np.asarray(e.fn(df)) if isinstance(e, Expr) else np.full(len(df._d), e)


class _Then:
    def __init__(self, cond, value):
        self.cond, self.value = cond, value

    def otherwise(self, other):
        c, a, b = self.cond, self.value, other
        name = a.name if isinstance(a, Expr) else "literal"
        return Expr(lambda df: pd.Series(np.where(np.asarray(c.fn(df), dtype=bool), _values(a, df), _values(b, df))),
                    name)


class _When:
    def __init__(self, cond):
        self.cond = cond

    def then(self, value):
        return _Then(self.cond, value)


def when(cond):
    return _When(cond)


def concat(frames):
    return DataFrame(pd.concat([f._d for f in frames], ignore_index=True))


class Series(list):
    def __init__(self, x, values=None):
        if isinstance(x, str):  # Series(name, values)
            self.name, x = x, values
        if isinstance(x, DataFrame):
            x = x._d.iloc[:, 0].tolist()
        super().__init__(x)

    def to_list(self):
        return list(self)

    def min(self):
        return min(self)

    def max(self):
        return max(self)


class _GroupBy:
    def __init__(self, df, key):
        self.df = df
        self.key = key

    def agg(self, *exprs):
        out = []
        for k, sub in self.df._d.groupby(self.key, sort=False):
            row = {self.key: k}
            sub_df = DataFrame(sub)
            for e in exprs:
                v = e.fn(sub_df)
                if e.agg == "unique":
                    row[e.name] = list(dict.fromkeys(v))
                elif e.agg == "max":
                    row[e.name] = v.max()
                else:
                    row[e.name] = v.iloc[0]
            out.append(row)
        return DataFrame(pd.DataFrame(out))


class DataFrame:
    def __init__(self, data=None, schema=None):
        if isinstance(data, pd.DataFrame):
            self._d = data.reset_index(drop=True)
            return
        if isinstance(data, dict):
            data = {k: (v if isinstance(v, list) else [v]) for k, v in data.items()}
        self._d = pd.DataFrame(data, columns=schema)

    @property
    def columns(self):
        return list(self._d.columns)

    def with_columns(self, *exprs):
        d = self._d.copy()
        for e in exprs:
            v = e.fn(self)
            d[e.name] = v.values if hasattr(v, "values") else v
        return DataFrame(d)

    def with_row_index(self, name="index"):
        d = self._d.copy()
        d.insert(0, name, range(len(d)))
        return DataFrame(d)

    def rename(self, mapping):
        return DataFrame(self._d.rename(columns=mapping))

    def drop(self, name):
        return DataFrame(self._d.drop(columns=[name]))

    def write_csv(self, path, separator=","):
        self._d.to_csv(path, sep=separator, index=False)

    def group_by(self, key, maintain_order=True):
        return _GroupBy(self, key)

    def get_column_index(self, name):
        return self.columns.index(name)

    def get_column(self, name):
        return Series(self._d[name].tolist())

    def __getitem__(self, name):
        return Series(self._d[name].tolist())

    def rows(self):
        return [tuple(r) for r in self._d.itertuples(index=False)]

    iter_rows = rows

    def join(self, other, on, how="left"):
        return DataFrame(self._d.merge(other._d, on=on, how=how))

    def filter(self, e):
        return DataFrame(self._d[np.asarray(e.fn(self), dtype=bool)])

    def sort(self, c):
        return DataFrame(self._d.sort_values(c.name if isinstance(c, Expr) else c, kind="stable"))

    def __len__(self):
        return len(self._d)

    def clone(self):
        return DataFrame(self._d.copy())

    def vstack(self, other):
        return DataFrame(pd.concat([self._d, other._d], ignore_index=True))

    def replace_column(self, index, series):
        d = self._d.copy()
        d[d.columns[index]] = list(series)
        return DataFrame(d)

    def __repr__(self):
        return repr(self._d)

    def item(self, row, column):
        v = self._d.iloc[row][column]
        return v.item() if hasattr(v, "item") else v

    def __setitem__(self, key, value):
        row, column = key
        self._d.at[self._d.index[row], column] = value


def read_csv(path, separator=","):
    return DataFrame(pd.read_csv(str(path), sep=separator))
