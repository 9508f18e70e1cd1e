"""Multi-GPU layer on CPU: world-size-2 gloo processes (127.0.0.1), the same
host logic bench.py runs on N GPUs over RCCL."""
import os
import socket
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_world_size_2_gloo():
    port = _free_port()
    procs = []
    for rank in range(2):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                   LOCAL_RANK=str(rank), CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "_dist_worker.py")], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out)
    for rank, (p, out) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, f"rank {rank} failed:\n{out}"
        assert f"ok rank {rank}" in out


def test_scan_order_key_query_order():
    """n_wg = 0 (a rows-step result): the pair hits come in query order."""
    import numpy as np

    from spectrseqtools_amd.parallel import scan_order_key

    q = np.array([5, 1, 9, 3])
    assert scan_order_key(q, 100, 0).tolist() == q.tolist()
