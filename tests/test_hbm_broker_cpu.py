"""The HBM broker's protocol on CPU: ``native/hbmbroker`` linked against the stub HIP runtime
(tests/native/fake_hip.c, whose exported VMM handles are memfds). Grants, takes, waiting in
arrival order, a container restart taking its grant again, timeouts, grant expiry, and hostile
input on both sockets. The real runtime is covered by tests/test_hbm_broker.py on MI355X."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import time

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GIB = 1 << 30


@pytest.fixture(scope="module")
def broker_exe(tmp_path_factory):
    d = tmp_path_factory.mktemp("fakehip-broker")
    lib = d / "libamdhip64.so.7"
    subprocess.run(["gcc", "-shared", "-fPIC", "-O1", "-Wl,-soname,libamdhip64.so.7", "-o", str(lib),
                    os.path.join(HERE, "native", "fake_hip.c")], check=True)
    exe = d / "gpushare-hbm-broker"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                    "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-o", str(exe),
                    os.path.join(ROOT, "native", "hbmbroker", "hbmbroker.cpp"), str(lib), f"-Wl,-rpath,{d}"],
                   check=True)
    return str(exe), str(d)


class Broker:
    def __init__(self, exe, path, gib=8, wait_s=1.0, ttl_s=600.0):
        exe, libdir = exe
        self.path = path
        env = dict(os.environ, LD_LIBRARY_PATH=libdir, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1",
                   UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
        self.p = subprocess.Popen([exe, "--socket", path, "--gib", str(gib), "--wait-s", str(wait_s),
                                   "--grant-ttl-s", str(ttl_s)], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                  text=True, env=env)
        assert json.loads(self.p.stdout.readline())["ready"]

    def admin(self, line):
        s = socket.socket(socket.AF_UNIX)
        s.settimeout(5)
        s.connect(self.path + ".admin")
        s.sendall(line.encode() + b"\n")
        out = b""
        while not out.endswith(b"\n"):
            c = s.recv(4096)
            if not c:
                break
            out += c
        s.close()
        return out.decode().strip()

    def stat(self):
        return json.loads(self.admin("STAT"))

    def stop(self):
        self.p.terminate()
        rc = self.p.wait(10)
        err = self.p.stderr.read()
        assert rc == 0 and "AddressSanitizer" not in err and "runtime error" not in err, err[-3000:]


class Pod:
    """A pod's shim side: TAKE, then the FDS header and the fds."""

    def __init__(self, path, token):
        self.s = socket.socket(socket.AF_UNIX)
        self.s.settimeout(10)
        self.s.connect(path)
        self.s.sendall(f"TAKE {token}\n".encode())

    def result(self):
        head = b""
        while not head.endswith(b"\n"):
            c = self.s.recv(1)
            if not c:
                return head.decode(), []
            head += c
        head = head.decode().strip()
        if not head.startswith("FDS "):
            return head, []
        n = int(head.split()[1])
        fds = []
        while len(fds) < n:
            _, got, _, _ = socket.recv_fds(self.s, 1, 200)
            fds += got
        for fd in fds:
            os.close(fd)
        return head, fds

    def close(self):
        self.s.close()


@pytest.fixture
def broker(broker_exe, tmp_path):
    b = Broker(broker_exe, str(tmp_path / "hbm0.sock"))
    yield b
    b.stop()


def test_grant_take_release_and_a_restart_takes_the_grant_again(broker):
    assert broker.admin(f"GRANT {'a' * 32} {5 * GIB + 1}") == "OK 6"          # rounded up to granules
    p = Pod(broker.path, "a" * 32)
    head, fds = p.result()
    assert head == f"FDS 6 {GIB}" and len(fds) == 6
    st = broker.stat()
    assert st["held"] == 6 and st["free"] == 2 and st["takes"] == 1
    again = Pod(broker.path, "a" * 32)          # a second process of the same pod: waits while held
    time.sleep(0.3)
    assert broker.stat()["waiting"] == 1
    p.close()                                    # the first process exits: scrubbed, then re-taken
    head, fds = again.result()
    assert head == f"FDS 6 {GIB}"
    st = broker.stat()
    assert st["releases"] == 1 and st["scrubbed_bytes"] >= 6 * GIB and st["takes"] == 2
    again.close()


def test_takes_wait_for_granules_in_arrival_order(broker):
    broker.admin(f"GRANT {'h' * 32} {6 * GIB}")
    broker.admin(f"GRANT {'w' * 32} {4 * GIB}")
    broker.admin(f"GRANT {'x' * 32} {1 * GIB}")
    holder = Pod(broker.path, "h" * 32)
    assert holder.result()[0] == f"FDS 6 {GIB}"
    first = Pod(broker.path, "w" * 32)           # needs 4 of the 2 free: waits
    time.sleep(0.1)
    second = Pod(broker.path, "x" * 32)          # would fit now, but does not overtake the first
    time.sleep(0.3)
    assert broker.stat()["waiting"] == 2
    holder.close()
    assert first.result()[0] == f"FDS 4 {GIB}"
    assert second.result()[0] == f"FDS 1 {GIB}"
    first.close()
    second.close()


def test_unknown_token_times_out_and_grants_expire(broker_exe, tmp_path):
    b = Broker(broker_exe, str(tmp_path / "hbm1.sock"), wait_s=0.5, ttl_s=0.5)
    try:
        p = Pod(b.path, "never")
        assert p.result()[0] == "ERR timeout"
        b.admin(f"GRANT {'e' * 32} {GIB}")
        time.sleep(1.0)
        st = b.stat()
        assert st["timeouts"] == 1 and st["expired"] == 1 and st["grants"] == 0
    finally:
        b.stop()


def test_hostile_input_ends_only_that_connection(broker):
    def send(path, data):
        s = socket.socket(socket.AF_UNIX)
        s.settimeout(5)
        s.connect(path)
        s.sendall(data)
        try:
            out = s.recv(256)
        except (socket.timeout, ConnectionResetError):
            out = b""
        s.close()
        return out

    assert send(broker.path, b"GRANT abc 999999999999\n").startswith(b"ERR")   # no grants from a pod
    assert send(broker.path, b"STAT\n").startswith(b"ERR")                     # nor its counters
    assert send(broker.path, b"\x00\xff garbage\n").startswith(b"ERR")
    assert send(broker.path, b"A" * 5000) == b""                               # over-long line: dropped
    assert send(broker.path + ".admin", b"GRANT t 0\n").startswith(b"ERR")     # no empty grants
    assert send(broker.path + ".admin", f"GRANT t {100 * GIB}\n".encode()).startswith(b"ERR")   # > the broker
    assert broker.stat()["refused"] >= 5
    broker.admin(f"GRANT {'k' * 32} {GIB}")                                    # still serving
    p = Pod(broker.path, "k" * 32)
    assert p.result()[0] == f"FDS 1 {GIB}"
    p.close()
    assert oct(os.stat(broker.path + ".admin").st_mode & 0o777) == "0o600"
