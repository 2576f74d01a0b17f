"""Frame-interleaved groups on the GPU: N member contexts
encode one stream, member k the frames n = k (mod N), and the result is the
single-context stream bit for bit (the multi-GPU protocol
emulated on one device).  Each case runs tests/group_worker.py in fresh
processes (the in-process group needs more hardware queues than the default
four; the cross-process group shares buffers through IPC handles)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "group_worker.py")


def _run(args, env=None, timeout=240):
    r = subprocess.run([sys.executable, WORKER] + [str(a) for a in args], capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    return r


@pytest.mark.parametrize("members,ring,w,h,frames,intra", [
    (2, 4, 352, 288, 14, 0),    # S = 2 slots per member, N * S == R: in place
    (3, 4, 352, 288, 15, 0),    # S = 2, N * S = 6 > R: out of place (stale rows from another member)
    (4, 4, 352, 288, 16, 5),    # one slot each, intra frames inside the stream
    (2, 2, 1280, 720, 8, 0),    # BASELINE configs[1] geometry
    (8, 4, 352, 288, 20, 0),    # eight members (the node's GPU count), S = 1 out of place
])
def test_group_in_process(members, ring, w, h, frames, intra):
    env = dict(os.environ, GPU_MAX_HW_QUEUES=str(min(32, 3 * members + 2)))
    r = _run(["inproc", "--members", members, "--ring", ring, "--w", w, "--h", h, "--frames", frames,
              "--intra-every", intra, "--batch", 3], env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["mismatched"] == []


def test_group_reset_rejoin():
    """Members reset (cairo_ctx_reset: tickets restart at 0) and rejoin, then
    encode the stream again from frame 0: their peers locate each member's
    output_cache and progress words by ticket, so both passes are bit-exact."""
    env = dict(os.environ, GPU_MAX_HW_QUEUES="8")
    r = _run(["inproc", "--members", 2, "--ring", 4, "--frames", 10, "--batch", 3, "--rejoin", 1], env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["mismatched"] == []


def test_group_in_process_refuses_few_queues():
    """Two in-process members under HIP's default 4 hardware queues would
    deadlock; join_group refuses with a diagnosis instead."""
    env = {k: v for k, v in os.environ.items() if k != "GPU_MAX_HW_QUEUES"}
    r = _run(["inproc", "--members", 2, "--ring", 4, "--frames", 4, "--batch", 2], env=env)
    assert r.returncode != 0
    assert "GPU_MAX_HW_QUEUES" in r.stderr


def test_group_4k_in_process():
    """BASELINE configs[3] geometry, two members, default launches."""
    env = dict(os.environ, GPU_MAX_HW_QUEUES="8")
    r = _run(["inproc", "--members", 2, "--ring", 4, "--w", 3840, "--h", 2160, "--frames", 6, "--batch", 16],
             env=env, timeout=280)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]


@pytest.mark.parametrize("members,feed,frames,size", [(2, False, 12, "cif"), (2, True, 12, "cif"), (3, True, 12, "cif"),
                                                      (4, True, 16, "cif"), (8, True, 20, "cif"), (2, True, 6, "4k")])
def test_group_cross_process(tmp_path, members, feed, frames, size):
    """One process per member on one device: buffers shared through IPC
    handles (fine-grained memory, system-scope hand-offs: the cross-GPU code
    path, each frame's deblock pushing it into the mirrors of the members
    that read it), records exchanged over gloo; with feed, the members hand
    over GPU-precoded feeds as bench.py's single-stream leg does, and every
    frame's payload is checked against the oracle's.  8 members: the node's
    GPU count (every frame pushed to R = 4 other members)."""
    store = tmp_path / "store"
    extra = ["--feed"] if feed else []
    if size == "4k":  # BASELINE configs[3] geometry with the library's 96 staging slots: 2.4 GB of
        extra += ["--w", "3840", "--h", "2160"]  # output_cache per member, imported in two chunks
    procs = [subprocess.Popen([sys.executable, WORKER, "xproc", "--members", str(members), "--rank", str(k), "--store",
                               str(store), "--frames", str(frames), "--batch", "3"] + extra, cwd=ROOT,
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for k in range(members)]
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=280)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, o, e))
    for rc, o, e in outs:
        assert rc == 0, o[-2000:] + e[-3000:]
