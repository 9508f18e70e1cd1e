"""Build record of libsstgpu.so: which sources (SHA-256), which compiler and
target, and the library's own SHA-256, written by the csrc Makefile after
every link.  The loader checks it (_native.load_library): a library whose
bytes or sources no longer match its record is refused, so a run can only
use the .so built from the tree it runs in.  usage: build_record.py write"""
import datetime
import hashlib
import json
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
HEADER = os.path.join(os.path.dirname(PKG), "include", "sst.h")
LIB = os.path.join(PKG, "libsstgpu.so")
RECORD = os.path.join(PKG, "build_record.json")
SOURCE_SUFFIXES = (".hip", ".cpp", ".h")


def sources():
    names = sorted(f for f in os.listdir(CSRC) if f.endswith(SOURCE_SUFFIXES))
    return [os.path.join(CSRC, f) for f in names] + [HEADER]


def sha256(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for block in iter(lambda: f.read(1 << 20), b""):
            h.update(block)
    return h.hexdigest()


def source_digests():
    return {os.path.relpath(p, os.path.dirname(PKG)): sha256(p) for p in sources()}


def write(lib=LIB, record=RECORD):
    try:
        hipcc = subprocess.run([os.environ.get("HIPCC", "/opt/rocm/bin/hipcc"), "--version"], capture_output=True,
                               text=True).stdout.splitlines()
    except OSError:
        hipcc = []
    rec = {"library": {"path": os.path.relpath(lib, os.path.dirname(PKG)), "sha256": sha256(lib),
                       "bytes": os.path.getsize(lib)},
           "sources": source_digests(),
           "compiler": [ln for ln in hipcc if ln.strip()][:2],
           "arch": os.environ.get("ARCH", "gfx950"),
           "built_at": datetime.datetime.now(datetime.timezone.utc).isoformat(timespec="seconds"),
           "mode": "make (spectrseqtools_amd/csrc/Makefile)"}
    with open(record, "w") as f:
        json.dump(rec, f, indent=1, sort_keys=True)


def check(lib=LIB, record=RECORD):
    """None when the library and the tree's sources match the record, else why not."""
    if not os.path.exists(record):
        return f"{record} is missing (built without the Makefile?)"
    with open(record) as f:
        rec = json.load(f)
    if sha256(lib) != rec["library"]["sha256"]:
        return "libsstgpu.so differs from the library its build record names"
    now = source_digests()
    changed = sorted(k for k in set(now) | set(rec["sources"]) if now.get(k) != rec["sources"].get(k))
    if changed:
        return f"sources changed since the library was built: {', '.join(changed)}"
    return None


if __name__ == "__main__" and sys.argv[1:] == ["write"]:
    write()
