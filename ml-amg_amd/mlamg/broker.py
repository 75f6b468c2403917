"""Opt-in amg_2_v broker: many worker processes, one GPU, unchanged callers (VERDICT r05 Next #4).

The reference farms grids over processes (ns/parallel/pool.py:139-186): every worker calls
`amg_2_v(A, P, b, x, ...)` once per grid (utils/train_dataset.py:114 with error_tol=1e-6,
utils/evaluate_dataset.py:96 with res_tol=1e-10). P processes each opening their own HIP context
on one GPU run P independent single solves. With MLAMG_BROKER=1 in the environment,
mlamg.multigrid.amg_2_v instead hands the call to ONE broker process per GPU, which coalesces the
calls that are pending at the same time into one fused launch (csrc/batch.hip, one workgroup
per problem: mlamg_amg2v_batch) — no caller edits.

* Start. The first call in any worker connects to the broker's Unix socket
  ($MLAMG_BROKER_DIR or the temp dir, mlamg-broker-<uid>-dev<d>.sock). If nobody listens, that
  worker starts the broker as a FRESH child process (subprocess.Popen of `python -m
  mlamg.broker --serve`, its own session; never an exec of a process that touched the GPU —
  the workers themselves never touch it) under a file lock, so one broker per GPU starts however
  many workers race. The broker exits after MLAMG_BROKER_IDLE seconds (default 120) without a
  connection, or on a shutdown request (shutdown()).
* Transfer. A request is a length-prefixed JSON header (parameters, array dtypes and shapes)
  followed by the raw bytes of A (indptr, indices, data), P (same), b and x over the socket; the
  answer carries x and the residual history the same way, and conv / iterations in the header.
* Batching. Each of the broker's batcher threads (MLAMG_BROKER_STREAMS, default 4, each with a
  HIP stream of its own, so a batch queued behind a slow one does not wait for it) takes every
  request queued at that moment, groups them by their keyword arguments and runs each group: the
  problems a single call would give the fused engine (n_c <= FUSED_SINGLE_MAX_NC) in one
  mlamg_amg2v_batch launch — each problem's path in the kernel follows its own size, so each
  result is bitwise its own single call (tests/test_gpu_batch.py, tests/test_gpu_broker.py) —
  and the others through the same amg_2_v a worker would call, one after another.
* Failure. A broker that dies (or closes the connection) makes the pending call raise
  BrokerError in the worker instead of hanging; the next call starts a new broker.
"""
from __future__ import annotations

import fcntl
import json
import os
import queue
import socket
import struct
import subprocess
import sys
import tempfile
import threading
import time

import numpy as np

ENV = "MLAMG_BROKER"
_HDR = struct.Struct("<Q")


class BrokerError(RuntimeError):
    """The broker could not be reached, died during the call, or reported an error."""


def enabled():
    return os.environ.get(ENV, "") not in ("", "0")


def device_index():
    return int(os.environ.get("MLAMG_BROKER_DEVICE", "0"))


def socket_path(device=None):
    d = os.environ.get("MLAMG_BROKER_DIR") or tempfile.gettempdir()
    dev = device_index() if device is None else device
    return os.path.join(d, f"mlamg-broker-{os.getuid()}-dev{dev}.sock")


# ---------------------------------------------------------------- framing
def _send_msg(sock, header, arrays=()):
    arrays = [np.ascontiguousarray(a) for a in arrays]
    header = dict(header, arrays=[[a.dtype.str, list(a.shape)] for a in arrays])
    h = json.dumps(header).encode()
    sock.sendall(_HDR.pack(len(h)) + h)
    for a in arrays:
        sock.sendall(memoryview(a).cast("B"))


def _recv_exact(sock, n):
    buf = bytearray(n)
    view = memoryview(buf)
    got = 0
    while got < n:
        k = sock.recv_into(view[got:], n - got)
        if k == 0:
            raise ConnectionError("connection closed")
        got += k
    return buf


def _recv_msg(sock):
    (n,) = _HDR.unpack(_recv_exact(sock, _HDR.size))
    header = json.loads(bytes(_recv_exact(sock, n)))
    arrays = []
    for dt, shape in header.get("arrays", []):
        dtype = np.dtype(dt)
        count = int(np.prod(shape)) if shape else 1
        raw = _recv_exact(sock, count * dtype.itemsize)
        arrays.append(np.frombuffer(raw, dtype=dtype).reshape(shape))
    return header, arrays


# ---------------------------------------------------------------- client
_client_lock = threading.Lock()
_client_sock = None
_client_pid = None


def _connect(path, timeout=None):
    s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    try:
        s.settimeout(timeout)
        s.connect(path)
        s.settimeout(None)
        return s
    except OSError:
        s.close()
        return None


def _start_broker(path):
    """Connect, starting the broker (a fresh child process) if nobody listens on `path`."""
    s = _connect(path)
    if s is not None:
        return s
    lock_path = path + ".lock"
    with open(lock_path, "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            s = _connect(path)  # another worker may have started it meanwhile
            if s is not None:
                return s
            pkg_root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
            env = dict(os.environ)
            env["PYTHONPATH"] = pkg_root + os.pathsep + env.get("PYTHONPATH", "")
            env.pop(ENV, None)  # the broker itself solves on the GPU
            log = open(path + ".log", "ab")
            subprocess.Popen([sys.executable, "-m", "mlamg.broker", "--serve", path,
                              "--device", str(device_index())],
                             stdin=subprocess.DEVNULL, stdout=log, stderr=log, env=env,
                             start_new_session=True, close_fds=True)
            log.close()
            deadline = time.monotonic() + float(os.environ.get("MLAMG_BROKER_START_S", "300"))
            while time.monotonic() < deadline:  # the first torch import on a fresh box is slow
                s = _connect(path)
                if s is not None:
                    return s
                time.sleep(0.05)
            raise BrokerError(f"the amg_2_v broker did not start (log: {path}.log)")
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)


def _request(header, arrays):
    """One call to the broker (one connection per worker process, reconnecting after a fork or
    a broker restart). Raises BrokerError if the broker is unreachable or dies meanwhile."""
    global _client_sock, _client_pid
    with _client_lock:
        if _client_sock is None or _client_pid != os.getpid():
            _client_sock = _start_broker(socket_path())
            _client_pid = os.getpid()
        s = _client_sock
        try:
            _send_msg(s, header, arrays)
            reply, out = _recv_msg(s)
        except (OSError, ConnectionError, ValueError) as e:
            try:
                s.close()
            finally:
                _client_sock = None
            raise BrokerError(f"amg_2_v broker connection lost: {e}") from None
    if not reply.get("ok"):
        raise BrokerError(f"amg_2_v broker: {reply.get('error', 'unknown error')}")
    return reply, out


def solve(A, P, b, x, params):
    """amg_2_v(A, P, b, x, **params) in the broker; the reference's return tuple."""
    import scipy.sparse as sp
    A = sp.csr_matrix(A)
    P = sp.csr_matrix(P)
    bv = np.ascontiguousarray(np.asarray(b, dtype=np.float64).ravel())
    xv = np.ascontiguousarray(np.asarray(x, dtype=np.float64).ravel())
    arrays = [A.indptr.astype(np.int32), A.indices.astype(np.int32), A.data.astype(np.float64),
              P.indptr.astype(np.int32), P.indices.astype(np.int32), P.data.astype(np.float64),
              bv, xv]
    header = {"op": "amg_2_v", "A_shape": list(A.shape), "P_shape": list(P.shape),
              "params": params}
    reply, out = _request(header, arrays)
    x_out, err, conv = out
    if reply.get("failed"):  # multigrid.py:167-170 returns the caller's own x
        return x, np.float64(1.), np.zeros(params.get("max_iter", 500)), 0
    return np.array(x_out), np.float64(conv[0]), np.array(err), int(reply["iters"])


def shutdown(device=None):
    """Ask a running broker to exit (no-op if none listens)."""
    s = _connect(socket_path(device), timeout=5)
    if s is None:
        return False
    try:
        _send_msg(s, {"op": "shutdown"})
        _recv_msg(s)
    except (OSError, ConnectionError):
        pass
    finally:
        s.close()
    return True


# ---------------------------------------------------------------- server
class _Server:
    def __init__(self, path, device, backend):
        self.path = path
        self.device = device
        self.backend = backend
        self.q = queue.Queue()
        self.stop = threading.Event()
        self.last_activity = time.monotonic()
        self.clients = 0
        self.lock = threading.Lock()
        self.stats = {"requests": 0, "batches": 0, "fused": 0, "single": 0}

    # one reader thread per connection
    def _serve_conn(self, conn):
        with self.lock:
            self.clients += 1
        try:
            while not self.stop.is_set():
                try:
                    header, arrays = _recv_msg(conn)
                except (ConnectionError, OSError, ValueError):
                    return
                if header.get("op") == "shutdown":
                    _send_msg(conn, {"ok": True})
                    self.stop.set()
                    return
                if header.get("op") == "stats":
                    _send_msg(conn, dict(self.stats, ok=True))
                    continue
                done = threading.Event()
                item = {"header": header, "arrays": arrays, "done": done}
                self.q.put(item)
                done.wait()
                try:
                    _send_msg(conn, item["reply"], item.get("out", ()))
                except OSError:
                    return
        finally:
            with self.lock:
                self.clients -= 1
                self.last_activity = time.monotonic()
            conn.close()

    def _batcher(self):
        ctx = None
        if self.backend is _gpu_backend:  # each batcher launches on a stream of its own, so a
            import torch                  # batch behind a slow one does not wait for it
            torch.cuda.set_device(self.device)
            ctx = torch.cuda.stream(torch.cuda.Stream(device=self.device))
        if ctx is not None:
            with ctx:
                self._batch_loop()
        else:
            self._batch_loop()

    def _batch_loop(self):
        while not self.stop.is_set():
            try:
                first = self.q.get(timeout=0.2)
            except queue.Empty:
                continue
            items = [first]
            while True:
                try:
                    items.append(self.q.get_nowait())
                except queue.Empty:
                    break
            with self.lock:
                self.stats["batches"] += 1
                self.stats["requests"] += len(items)
            try:
                self.backend(self, items)
            except Exception as e:  # every waiting worker gets the error, none hangs
                for it in items:
                    if "reply" not in it:
                        it["reply"] = {"ok": False, "error": f"{type(e).__name__}: {e}"}
            for it in items:
                if "reply" not in it:
                    it["reply"] = {"ok": False, "error": "no result"}
                it["done"].set()

    def run(self):
        try:
            os.unlink(self.path)
        except FileNotFoundError:
            pass
        srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        srv.bind(self.path)
        os.chmod(self.path, 0o600)  # this user's workers only
        srv.listen(256)
        with open(self.path + ".pid", "w") as fh:
            fh.write(str(os.getpid()))
        srv.settimeout(0.5)
        for i in range(max(1, int(os.environ.get("MLAMG_BROKER_STREAMS", "4")))):
            threading.Thread(target=self._batcher, daemon=True,
                             name=f"mlamg-broker-batch{i}").start()
        idle = float(os.environ.get("MLAMG_BROKER_IDLE", "120"))
        try:
            while not self.stop.is_set():
                try:
                    conn, _ = srv.accept()
                except socket.timeout:
                    with self.lock:
                        if self.clients == 0 and time.monotonic() - self.last_activity > idle:
                            break
                    continue
                with self.lock:
                    self.last_activity = time.monotonic()
                threading.Thread(target=self._serve_conn, args=(conn,), daemon=True).start()
        finally:
            srv.close()
            for f in (self.path, self.path + ".pid"):
                try:
                    os.unlink(f)
                except FileNotFoundError:
                    pass


def _unpack(item):
    import scipy.sparse as sp
    h, a = item["header"], item["arrays"]
    A = sp.csr_matrix((a[2], a[1], a[0]), shape=tuple(h["A_shape"]))
    P = sp.csr_matrix((a[5], a[4], a[3]), shape=tuple(h["P_shape"]))
    return A, P, np.array(a[6]), np.array(a[7]), h["params"]


def _answer(item, res, x_in):
    x, conv, err, iters = res
    item["reply"] = {"ok": True, "iters": int(iters), "failed": x is x_in}
    item["out"] = [np.asarray(x, dtype=np.float64), np.asarray(err, dtype=np.float64),
                   np.array([conv], dtype=np.float64)]


def _gpu_backend(server, items):
    """Group by keyword arguments; fused-kernel problems of a group in one launch, the rest as
    the single calls a worker would make."""
    from . import multigrid as mg
    groups = {}
    for it in items:
        try:
            A, P, b, x, params = _unpack(it)
        except Exception as e:
            it["reply"] = {"ok": False, "error": f"bad request: {e}"}
            continue
        key = json.dumps(params, sort_keys=True)
        groups.setdefault(key, []).append((it, A, P, b, x, params))
    for members in groups.values():
        params = members[0][5]
        kw = dict(pre_smoothing_steps=1, post_smoothing_steps=1, jacobi_weight=0.666,
                  res_tol=None, error_tol=None, max_iter=500, singular=False,
                  smoother="gauss_seidel")
        kw.update(params)
        fused, prepared, xs = [], [], []
        if not kw["singular"]:
            for m in members:
                # every problem a single call would give the fused engine (n_c up to
                # FUSED_SINGLE_MAX_NC): its path inside the kernel follows its own n_c, so the
                # batch result is its single call's, bit for bit (tests/test_gpu_broker.py)
                prep = mg._fused_arrays(m[1], m[2], m[3], m[4], mg.FUSED_SINGLE_MAX_NC)
                if prep is not None:
                    fused.append(m)
                    prepared.append(prep)
                    xs.append(m[4])
        out = None
        if prepared:
            out = mg._amg_2_v_fused(prepared, xs, kw["pre_smoothing_steps"],
                                    kw["post_smoothing_steps"], kw["jacobi_weight"],
                                    kw["res_tol"], kw["error_tol"], kw["max_iter"],
                                    kw["smoother"])
        done = set()
        if out is not None:
            server.stats["fused"] += len(fused)
            for m, res in zip(fused, out):
                _answer(m[0], res, m[4])
                done.add(id(m[0]))
        for m in members:
            if id(m[0]) in done:
                continue
            it, A, P, b, x, _ = m
            try:
                res = mg.amg_2_v(A, P, b, x, **params)
                server.stats["single"] += 1
                _answer(it, res, x)
            except Exception as e:
                it["reply"] = {"ok": False, "error": f"{type(e).__name__}: {e}"}


def _test_backend(server, items):
    """MLAMG_BROKER_BACKEND=test-hold (tests/test_broker.py only, no GPU): requests are held
    until the broker is killed, to check that a worker then gets an error instead of hanging;
    test-echo returns x unchanged with one history entry."""
    mode = os.environ.get("MLAMG_BROKER_BACKEND")
    if mode == "test-hold":
        time.sleep(3600)
    for it in items:
        x = np.array(it["arrays"][7])
        _answer(it, (x, np.float64(0.5), np.array([1.0]), 1), None)


def serve(path, device):
    backend = _gpu_backend
    if os.environ.get("MLAMG_BROKER_BACKEND", "").startswith("test-"):
        backend = _test_backend
    else:
        import torch
        torch.cuda.set_device(device)
    _Server(path, device, backend).run()


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--serve", required=True)
    ap.add_argument("--device", type=int, default=0)
    a = ap.parse_args()
    serve(a.serve, a.device)
