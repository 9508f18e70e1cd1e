"""Diagnostic: the skeleton alphabet of one reference spectrum on the device."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "tests"), os.path.join(HERE, "..")]
import numpy as np  # noqa: E402

import _callers_checks as C  # noqa: E402
from conftest import load_golden  # noqa: E402
from spectrseqtools_amd import _native, pipeline, pipeline_device as PD  # noqa: E402

eng = _native.get_engine(0)
rec = load_golden("callers.json.gz")[sys.argv[1]]
dp = C.make_dp(rec["ctx"], engine=eng)
rows, fx, sk = C.device_pipeline_skeleton(rec, dp)
N = len(dp.masses)
b = PD.bins_device(dp, rows, fx.alpha)
print("fx.alpha rows", np.flatnonzero(pipeline.mask_rows(fx.alpha, N)[0]).tolist())
print("alpha_dev rows", np.flatnonzero(pipeline.mask_rows(b.alpha_dev.cpu().numpy().view(np.uint64), N)[0]).tolist())
ml = int(sk.max_len[0])
skel = sk.skel[:2 * ml].cpu().numpy().view(np.uint64)
u = np.zeros(2, np.uint64)
for p in skel:
    u |= p
print("U rows", np.flatnonzero(pipeline.mask_rows(u[None, :], N)[0]).tolist())
ln = PD.length_device(dp, sk, b.alpha_dev, [dp.seq.su_mass], [dp.seq.obs_mass])
print("alpha_sk rows", np.flatnonzero(pipeline.mask_rows(ln.alpha, N)[0]).tolist())
print("is_mod", [r for r in range(N) if dp.masses[r].is_modification][:10])
print("skel_off", sk.skel_off, "max_len", sk.max_len, "skel shape", tuple(sk.skel.shape))
