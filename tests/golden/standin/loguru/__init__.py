"""Import-only stand-in for `loguru` (absent from this image).

TEST INFRASTRUCTURE ONLY: put on sys.path by tests/golden/make_callers_golden.py
so the reference's prediction.py / skeleton_building.py import unmodified.
The reference only calls logger.warning (skeleton_building.py:165-171,
prediction.py:149-156); messages are kept in `logger.records`."""


class _Logger:
    def __init__(self):
        self.records = []

    def _log(self, level, msg, *args, **kwargs):
        self.records.append((level, str(msg)))

    def warning(self, msg, *args, **kwargs):
        self._log("WARNING", msg)

    def info(self, msg, *args, **kwargs):
        self._log("INFO", msg)

    def debug(self, msg, *args, **kwargs):
        self._log("DEBUG", msg)

    def error(self, msg, *args, **kwargs):
        self._log("ERROR", msg)


logger = _Logger()
