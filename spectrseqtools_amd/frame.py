"""A minimal column frame standing in for the polars DataFrames the hot path
reads (EXPLANATION_MASSES and the nucleotide_df handed to
DynamicProgrammingTable).  Only read access plus the two updates callers make
(alphabet / modification-rate edits) are provided.  Any object with
`get_column(name).to_list()` -- e.g. a real polars DataFrame -- is accepted
wherever a Frame is.
"""


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

    __getitem__ = get_column

    def get_column_index(self, name):
        return self.columns.index(name)

    def rows(self):
        return list(zip(*self._cols.values()))

    iter_rows = rows

    def filter_rows(self, predicate):
        keep = [i for i, r in enumerate(self.rows()) if predicate(dict(zip(self.columns, r)))]
        return Frame({k: [v[i] for i in keep] for k, v in self._cols.items()})

    def sort(self, name):
        order = sorted(range(len(self)), key=lambda i: self._cols[name][i])
        return Frame({k: [v[i] for i in order] for k, v in self._cols.items()})

    def with_column(self, name, values):
        cols = dict(self._cols)
        cols[name] = list(values)
        return Frame(cols)

    def with_modification_rates(self, rate_of):
        """New frame whose modification_rate column is rate_of(row_dict) -- the
        cli's singleton / canonical-base rate edits (cli.py:115-139)."""
        rates = [rate_of(dict(zip(self.columns, r))) for r in self.rows()]
        return self.with_column("modification_rate", rates)

    def __repr__(self):
        return f"Frame({len(self)} rows: {', '.join(self.columns)})"
