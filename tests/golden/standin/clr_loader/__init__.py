"""Import-only stand-in for `clr_loader` (absent; the .NET RAW reader is out of
scope).  TEST INFRASTRUCTURE ONLY: common.py calls get_mono() at import."""


def get_mono(*args, **kwargs):
    return None
