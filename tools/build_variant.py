"""Build an experimental variant of libsstgpu.so for tools/ab_bench.sh:
copies spectrseqtools_amd/csrc to a scratch dir, applies literal
(old -> new) replacements from a JSON file, and compiles with the Makefile's
flags into build/ab/<name>.so.  usage: build_variant.py NAME EDITS.json"""
import json
import os
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
name, edits = sys.argv[1], json.load(open(sys.argv[2]))
tmp = tempfile.mkdtemp()
src = os.path.join(tmp, "csrc")
shutil.copytree(os.path.join(REPO, "spectrseqtools_amd", "csrc"), src)
for fname, pairs in edits.items():
    p = os.path.join(src, fname)
    s = open(p).read()
    for old, new in pairs:
        if old not in s:
            sys.exit(f"{name}: edit not found in {fname}: {old[:60]!r}")
        s = s.replace(old, new)
    open(p, "w").write(s)
out = os.path.join(REPO, "build", "ab", name + ".so")
os.makedirs(os.path.dirname(out), exist_ok=True)
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
                "-fno-fast-math", "-DSST_DIAG", "-I" + os.path.join(REPO, "include"), "-I" + src, "-shared", "-o", out,
                *[os.path.join(src, f) for f in ("sst_kernels.hip", "sst_alpha.hip", "sst_rows.hip", "sst_pipe.hip",
                                                  "sst_skel.hip", "sst_reach.hip", "sst_frontier.hip", "sst_api.cpp")]],
               check=True)
shutil.rmtree(tmp)
print(out)
