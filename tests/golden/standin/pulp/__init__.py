"""Import-only stand-in for `pulp` (absent from this image; the MILP is out of
scope).  TEST INFRASTRUCTURE ONLY: lets linear_program.py import so that
prediction.py and skeleton_building.py load; every name refuses to be used,
so no fixture can silently depend on a solver."""


class _Unavailable:
    def __init__(self, *args, **kwargs):
        raise NotImplementedError("pulp stand-in: the MILP is not available in this container")


class LpProblem(_Unavailable):
    pass


class LpVariable(_Unavailable):
    pass


LpMinimize = 1
LpMaximize = -1
LpInteger = "Integer"
LpContinuous = "Continuous"
LpBinary = "Binary"


def lpSum(*args, **kwargs):
    raise NotImplementedError("pulp stand-in: the MILP is not available in this container")


def getSolver(*args, **kwargs):
    raise NotImplementedError("pulp stand-in: the MILP is not available in this container")
