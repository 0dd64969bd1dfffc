"""The HBM broker's protocol on CPU: ``native/hbmbroker`` linked against the stub HIP runtime
(tests/native/fake_hip.c, whose exported VMM handles are memfds and whose events complete after
``FAKE_HIP_EVENT_MS``). Grants, takes, waiting in arrival order, a container restart taking its
grant again, timeouts, REVOKE / LIST / boot id, the admin socket apart from the pod socket, caps
on junk connections, scrubs that do not stall the event loop, the release policies, and hostile
input on both sockets. The real runtime is covered by tests/test_hbm_broker.py on MI355X."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys
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


def _line(path, line, timeout=5.0):
    s = socket.socket(socket.AF_UNIX)
    s.settimeout(timeout)
    s.connect(path)
    s.sendall(line.encode() + b"\n")
    out = b""
    while not out.endswith(b"\n"):
        c = s.recv(65536)
        if not c:
            break
        out += c
    s.close()
    return out.decode().strip()


class Broker:
    def __init__(self, exe, path, gib=8, wait_s=1.0, ttl_s=0.0, policy="trust", admin=None, extra=(), env=None):
        exe, libdir = exe
        self.path = path
        self.admin_path = admin or path + ".admin"
        env = dict(os.environ, LD_LIBRARY_PATH=libdir, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1",
                   UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", **(env or {}))
        self.p = subprocess.Popen([exe, "--socket", path, "--admin-socket", self.admin_path, "--gib", str(gib),
                                   "--wait-s", str(wait_s), "--grant-ttl-s", str(ttl_s), "--release-policy", policy,
                                   *extra], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
        self.ready = json.loads(self.p.stdout.readline())
        assert self.ready["ready"]

    def admin(self, line):
        return _line(self.admin_path, line)

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
        if head.split(" ")[0] not in ("FDS", "MORE", "XFDS"):
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


class StreamPod(Pod):
    """A streaming TAKE: the first answer at once, the rest in MORE batches."""

    def __init__(self, path, token):
        self.s = socket.socket(socket.AF_UNIX)
        self.s.settimeout(10)
        self.s.connect(path)
        self.s.sendall(f"TAKE {token} STREAM\n".encode())

    def more(self, timeout=5.0):
        self.s.settimeout(timeout)
        try:
            return self.result()
        finally:
            self.s.settimeout(10)


def test_streaming_take_gets_what_is_free_at_once_and_the_rest_as_it_comes_back(broker):
    broker.admin(f"GRANT {'h' * 32} {6 * GIB}")
    broker.admin(f"GRANT {'s' * 32} {4 * GIB}")
    broker.admin(f"GRANT {'p' * 32} {1 * GIB}")
    broker.admin(f"GRANT {'q' * 32} {1 * GIB}")
    holder = Pod(broker.path, "h" * 32)
    assert holder.result()[0] == f"FDS 6 {GIB}"
    t = time.perf_counter()
    st = StreamPod(broker.path, "s" * 32)
    head, fds = st.result()
    assert head == f"FDS 2 {GIB} 4 4" and len(fds) == 2 and time.perf_counter() - t < 1.0   # no wait
    plain = Pod(broker.path, "p" * 32)           # arrives later: waits behind the streamer's owed 2
    time.sleep(0.1)
    late = StreamPod(broker.path, "q" * 32)      # a later streamer is accepted with nothing yet
    assert late.result()[0] == f"FDS 0 {GIB} 1 1"
    s = broker.stat()
    assert s["owed"] == 2 + 1 and s["waiting"] == 1 and s["streamed"] == 2 and s["free"] == 0
    holder.close()                               # 6 back: 2 owed to the streamer, then the plain 1, then 1 owed
    assert st.more()[0] == f"MORE 2 {GIB}"
    assert plain.result()[0] == f"FDS 1 {GIB}"
    assert late.more()[0] == f"MORE 1 {GIB}"
    s = broker.stat()
    assert s["owed"] == 0 and s["held"] == 4 + 1 + 1 and s["free"] == 2 and s["more_msgs"] == 2
    for p in (st, plain, late):
        p.close()


@pytest.mark.parametrize("chunk", [2, 0])
def test_a_released_pods_granules_are_lent_as_their_scrub_progresses(broker_exe, tmp_path, chunk):
    """The broker zeroes a released pod's granules in chunks (--scrub-chunk, an event each): a
    streaming taker gets the first ones once their chunk is zeroed, not after the whole release.
    The stub GPU zeroes 100 ms per granule here; 6 granules come back, 4 are owed."""
    b = Broker(broker_exe, str(tmp_path / "hbm0.sock"), extra=("--scrub-chunk", str(chunk)),
               env={"FAKE_HIP_MEMSET_MS_PER_GIB": "100"})
    try:
        b.admin(f"GRANT {'h' * 32} {6 * GIB}")
        b.admin(f"GRANT {'s' * 32} {6 * GIB}")
        holder = Pod(b.path, "h" * 32)
        assert holder.result()[0] == f"FDS 6 {GIB}"
        st = StreamPod(b.path, "s" * 32)
        assert st.result()[0] == f"FDS 2 {GIB} 6 6"
        t0 = time.perf_counter()
        holder.close()
        got = []
        while sum(n for n, _ in got) < 4:
            head = st.more()[0]
            got.append((int(head.split()[1]), time.perf_counter() - t0))
        if chunk:
            assert [n for n, _ in got] == [2, 2] and got[0][1] < 0.35 and 0.35 < got[1][1] < 0.8, got
        else:
            assert [n for n, _ in got] == [4] and got[0][1] > 0.55, got
        st.close()
    finally:
        b.stop()


def test_a_streamer_that_leaves_while_owed_frees_its_place(broker):
    """A streaming taker owed granules goes away: what it held is returned and scrubbed, what it
    was owed is forgotten, and the next taker in line is served."""
    broker.admin(f"GRANT {'h' * 32} {6 * GIB}")
    broker.admin(f"GRANT {'s' * 32} {5 * GIB}")
    broker.admin(f"GRANT {'n' * 32} {2 * GIB}")
    holder = Pod(broker.path, "h" * 32)
    assert holder.result()[0] == f"FDS 6 {GIB}"
    st = StreamPod(broker.path, "s" * 32)
    assert st.result()[0] == f"FDS 2 {GIB} 5 5"
    nxt = Pod(broker.path, "n" * 32)                 # a plain TAKE of 2, behind the streamer's owed 3
    time.sleep(0.2)
    assert broker.stat()["owed"] == 3 and broker.stat()["waiting"] == 1
    st.close()                                       # gone while owed: its 2 come back, its 3 are forgotten
    assert nxt.result()[0] == f"FDS 2 {GIB}"
    s = broker.stat()
    assert s["owed"] == 0 and s["held"] == 6 + 2
    holder.close()
    nxt.close()


def test_a_revoked_streamer_is_sent_no_more(broker):
    broker.admin(f"GRANT {'h' * 32} {7 * GIB}")
    broker.admin(f"GRANT {'r' * 32} {4 * GIB}")
    holder = Pod(broker.path, "h" * 32)
    assert holder.result()[0] == f"FDS 7 {GIB}"
    st = StreamPod(broker.path, "r" * 32)
    assert st.result()[0] == f"FDS 1 {GIB} 4 4"
    assert broker.admin(f"REVOKE {'r' * 32}") == "OK 1"
    assert st.more(timeout=2)[0] == "END"            # told: the shim ends its stream at what it has
    holder.close()
    with pytest.raises(TimeoutError):
        st.more(timeout=0.5)
    s = broker.stat()
    assert s["owed"] == 0 and s["held"] == 1
    st.close()
    time.sleep(0.2)
    assert broker.stat()["held"] == 0


def test_ungranted_take_gets_a_short_deadline_and_a_late_grant_is_served(broker_exe, tmp_path):
    b = Broker(broker_exe, str(tmp_path / "hbm1.sock"), wait_s=30.0, extra=("--ungranted-wait-s", "0.5"))
    try:
        t = time.monotonic()
        assert Pod(b.path, "never").result()[0] == "ERR nogrant"               # not the 30 s of --wait-s
        assert time.monotonic() - t < 3.0
        p = Pod(b.path, "l" * 32)                                             # the grant comes after the TAKE
        time.sleep(0.2)
        assert b.admin(f"GRANT {'l' * 32} {GIB}") == "OK 1"
        assert p.result()[0] == f"FDS 1 {GIB}"
        p.close()
        st = b.stat()
        assert st["timeouts"] == 1 and st["takes"] == 1
    finally:
        b.stop()


def test_grants_expire_only_with_a_ttl(broker_exe, tmp_path):
    b = Broker(broker_exe, str(tmp_path / "hbm1.sock"), ttl_s=0.5)
    try:
        b.admin(f"GRANT {'e' * 32} {GIB}")
        time.sleep(1.0)
        st = b.stat()
        assert st["expired"] == 1 and st["grants"] == 0
    finally:
        b.stop()
    b = Broker(broker_exe, str(tmp_path / "hbm2.sock"))                     # default: no TTL
    try:
        b.admin(f"GRANT {'e' * 32} {GIB}")
        time.sleep(0.5)
        assert b.stat()["grants"] == 1
    finally:
        b.stop()


def test_revoke_list_and_boot_id(broker_exe, tmp_path):
    b = Broker(broker_exe, str(tmp_path / "hbm0.sock"))
    try:
        boot = b.ready["boot"]
        assert len(boot) == 16 and b.stat()["boot"] == boot
        b.admin(f"GRANT {'r' * 32} {2 * GIB}")
        b.admin(f"GRANT {'s' * 32} {GIB}")
        assert json.loads(b.admin("LIST")) == {"boot": boot, "grants": {"r" * 32: 2, "s" * 32: 1}}
        held = Pod(b.path, "r" * 32)
        assert held.result()[0] == f"FDS 2 {GIB}"
        waiter = Pod(b.path, "r" * 32)                   # a second process of the pod waits ...
        time.sleep(0.2)
        assert b.admin(f"REVOKE {'r' * 32}") == "OK 2"   # ... the pod is deleted: 2 granules still held
        assert waiter.result()[0] == "ERR revoked"
        assert Pod(b.path, "r" * 32).result()[0] == "ERR revoked"   # never taken again
        assert json.loads(b.admin("LIST"))["grants"] == {"s" * 32: 1}
        held.close()                                     # the holder exits: the granules come back
        time.sleep(0.3)
        st = b.stat()
        assert st["free"] == 8 and st["held"] == 0 and st["revokes"] == 1 and st["revoked"] == 1
        assert b.admin(f"REVOKE {'z' * 32}") == "OK 0"   # unknown tokens are revoked too
        assert b.admin(f"GRANT {'r' * 32} {GIB}") == "OK 1"   # the granter may grant it again
        p = Pod(b.path, "r" * 32)
        assert p.result()[0] == f"FDS 1 {GIB}"
        p.close()
    finally:
        b.stop()
    b2 = Broker(broker_exe, str(tmp_path / "hbm0.sock"))     # a restart: a new boot id, no grants
    try:
        assert b2.ready["boot"] != boot and json.loads(b2.admin("LIST"))["grants"] == {}
    finally:
        b2.stop()


def test_admin_socket_lives_apart_and_checks_the_peer(broker_exe):
    import pathlib
    import tempfile

    root = pathlib.Path(tempfile.mkdtemp(prefix="gs-peer-", dir="/tmp"))   # reachable by another uid
    os.chmod(root, 0o755)
    pods = root / "gpu0"
    adm = root / "admin"
    pods.mkdir()
    adm.mkdir(mode=0o700)
    b = Broker(broker_exe, str(pods / "hbm0.sock"), admin=str(adm / "hbm0.sock"))
    try:
        assert sorted(os.listdir(pods)) == ["hbm0.sock"]                 # what a container mounts
        assert oct(os.stat(adm / "hbm0.sock").st_mode & 0o777) == "0o600"
        assert oct(os.stat(pods / "hbm0.sock").st_mode & 0o777) == "0o666"
        assert b.admin(f"GRANT {'k' * 32} {GIB}") == "OK 1"               # root: accepted
        if os.geteuid() == 0:
            # another uid that reaches the socket anyway (mode opened up) is refused by SO_PEERCRED
            os.chmod(adm / "hbm0.sock", 0o666)
            os.chmod(adm, 0o755)
            code = ("import socket,sys,time\ns=socket.socket(socket.AF_UNIX); s.connect(sys.argv[1]); time.sleep(0.2)\n"
                    "try: s.sendall(b'GRANT " + "q" * 32 + " 1073741824\\n')\nexcept OSError: pass\n"
                    "print(s.recv(64).decode().strip())")
            out = subprocess.run([sys.executable, "-c", code, str(adm / "hbm0.sock")], capture_output=True, text=True,
                                 user=65534, timeout=30)
            assert out.stdout.strip() == "ERR peer", out
            assert b.stat()["peer_refused"] == 1 and json.loads(b.admin("LIST"))["grants"] == {"k" * 32: 1}
    finally:
        b.stop()


def test_junk_connections_do_not_delay_a_take(broker_exe, tmp_path):
    """1,000 connections that never ask anything: the per-peer cap turns nearly all of them away
    at once, the rest are dropped at the request deadline, and a legitimate TAKE from another
    process is served within 50 ms meanwhile."""
    b = Broker(broker_exe, str(tmp_path / "hbm0.sock"), extra=("--request-timeout-s", "1"))
    try:
        b.admin(f"GRANT {'t' * 32} {GIB}")
        junk, connected = [], 0
        for _ in range(1000):
            s = socket.socket(socket.AF_UNIX)
            s.setblocking(False)
            try:
                s.connect(b.path)
                connected += 1
            except (BlockingIOError, ConnectionRefusedError, OSError):
                pass                                   # the listen backlog is full: refused by the kernel
            junk.append(s)
        time.sleep(0.3)
        code = ("import socket,sys,time; t=time.perf_counter(); s=socket.socket(socket.AF_UNIX); "
                "s.connect(sys.argv[1]); s.sendall(('TAKE '+'t'*32+'\\n').encode()); h=b''\n"
                "while not h.endswith(b'\\n'): h+=s.recv(1)\n"
                "print(h.decode().strip(), round((time.perf_counter()-t)*1e3,2))")
        out = subprocess.run([sys.executable, "-c", code, b.path], capture_output=True, text=True, timeout=30)
        head, ms = out.stdout.split()[:3], float(out.stdout.split()[-1])
        assert " ".join(head) == f"FDS 1 {GIB}", out
        assert ms < 50.0, ms
        st = b.stat()
        assert connected >= 200 and st["busy"] >= connected - 8 and st["clients"] <= 8 + 2
        time.sleep(1.5)
        assert b.stat()["idle_dropped"] >= 1
        for s in junk:
            s.close()
    finally:
        b.stop()


def test_scrub_in_flight_does_not_stall_grant_take_or_stat(broker_exe, tmp_path):
    """A release's scrub takes 1.5 s on the stub GPU (FAKE_HIP_EVENT_MS): GRANT, STAT and a TAKE
    of free granules are answered meanwhile; the scrubbed granules come back after it."""
    b = Broker(broker_exe, str(tmp_path / "hbm0.sock"), wait_s=10.0, env={"FAKE_HIP_EVENT_MS": "1500"})
    try:
        b.admin(f"GRANT {'a' * 32} {6 * GIB}")
        p = Pod(b.path, "a" * 32)
        assert p.result()[0] == f"FDS 6 {GIB}"
        p.close()
        time.sleep(0.1)
        t = time.perf_counter()
        st = b.stat()
        assert st["scrubbing"] == 6 and st["free"] == 2
        assert b.admin(f"GRANT {'b' * 32} {2 * GIB}") == "OK 2"
        q = Pod(b.path, "b" * 32)
        assert q.result()[0] == f"FDS 2 {GIB}"
        assert time.perf_counter() - t < 0.5
        r = Pod(b.path, "a" * 32)                          # needs the granules being scrubbed: waits
        assert r.result()[0] == f"FDS 6 {GIB}"
        assert time.perf_counter() - t > 1.0
        st = b.stat()
        assert st["scrubbing"] == 0 and st["scrubbed_bytes"] >= 6 * GIB
        q.close()
        r.close()
    finally:
        b.stop()


def test_exit_policy_lends_only_after_the_holder_exits(broker_exe, tmp_path):
    """Release policy "exit" (the default where the kernel does not count dma-buf references, as
    with the stub's memfds): a holder that closes its connection but keeps running does not get
    its granules lent to the next pod; they are lent once its process has exited."""
    b = Broker(broker_exe, str(tmp_path / "hbm0.sock"), gib=2, policy="auto")
    try:
        assert b.ready["release_policy"] == "exit"
        b.admin(f"GRANT {'o' * 32} {2 * GIB}")
        b.admin(f"GRANT {'n' * 32} {2 * GIB}")
        code = ("import socket,sys,time; s=socket.socket(socket.AF_UNIX); s.connect(sys.argv[1]); "
                "s.sendall(('TAKE '+'o'*32+'\\n').encode()); h=b''\n"
                "while not h.endswith(b'\\n'): h+=s.recv(1)\n"
                "socket.recv_fds(s,1,200); s.close(); print('released', flush=True); sys.stdin.read()")
        tenant = subprocess.Popen([sys.executable, "-c", code, b.path], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                  text=True)
        assert tenant.stdout.readline().strip() == "released"      # connection closed, process alive
        nxt = Pod(b.path, "n" * 32)
        time.sleep(0.5)
        st = b.stat()
        assert st["quarantined"] == 2 and st["waiting"] == 1 and st["free"] == 0
        tenant.stdin.close()
        tenant.wait(10)
        assert nxt.result()[0] == f"FDS 2 {GIB}"
        nxt.close()
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
    assert send(broker.path, b"LIST\n").startswith(b"ERR")                     # nor the tokens
    assert send(broker.path, b"REVOKE abc\n").startswith(b"ERR")               # nor revocations
    assert send(broker.path, b"\x00\xff garbage\n").startswith(b"ERR")
    assert send(broker.path, b"TAKE ../../etc\n").startswith(b"ERR")           # tokens are [A-Za-z0-9_-]
    assert send(broker.path, b"A" * 5000) == b""                               # over-long line: dropped
    adm = broker.admin_path
    assert send(adm, b"GRANT t 0\n").startswith(b"ERR")                        # no empty grants
    assert send(adm, f"GRANT t {100 * GIB}\n".encode()).startswith(b"ERR")    # > the broker
    # bytes near 2^64 must not wrap into a small grant when rounded up to granules
    assert send(adm, b"GRANT t 18446744073709551615\n").startswith(b"ERR size")
    assert send(adm, b"GRANT t 18446744073709551000\n").startswith(b"ERR size")
    assert send(adm, b"GRANT t 1 extra\n").startswith(b"ERR")
    assert broker.stat()["refused"] >= 9
    broker.admin(f"GRANT {'k' * 32} {GIB}")                                    # still serving
    p = Pod(broker.path, "k" * 32)
    assert p.result()[0] == f"FDS 1 {GIB}"
    p.close()
    assert oct(os.stat(adm).st_mode & 0o777) == "0o600"


def test_a_sized_broker_grows_while_memory_comes_back_and_streams_grants_meanwhile(broker_exe, tmp_path):
    """--gib N right after another process freed its memory (amdgpu still wiping it; the stub
    holds 8 of 16 GiB for 1.5 s): the broker starts with what is free less a 2 GiB margin, grows to
    N as the memory comes back, accepts grants up to N at once, and a streaming TAKE gets its
    granules as they are created."""
    exe, libdir = broker_exe
    env = dict(os.environ, LD_LIBRARY_PATH=libdir, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1",
               FAKE_HIP_TOTAL_GIB="16", FAKE_HIP_HELD_GIB="8", FAKE_HIP_HELD_MS="1500")
    path = str(tmp_path / "hbm0.sock")
    p = subprocess.Popen([exe, "--socket", path, "--gib", "10", "--release-policy", "trust"],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
    try:
        ready = json.loads(p.stdout.readline())
        assert ready["granules"] == 6                       # 16 - 8 held - 2 margin
        assert _line(path + ".admin", f"GRANT {'g' * 32} {9 * GIB}") == "OK 9"     # up to the full 10
        assert _line(path + ".admin", f"GRANT {'x' * 32} {11 * GIB}") == "ERR size"
        pod = StreamPod(path, "g" * 32)
        assert pod.result()[0] == f"FDS 6 {GIB} 9 9"
        head = pod.more(timeout=10)[0]                      # the rest once grown and zeroed
        assert head == f"MORE 3 {GIB}", head
        st = json.loads(_line(path + ".admin", "STAT"))
        assert st["granules"] == 10 and st["grown"] == 4 and st["owed"] == 0, st
        pod.close()
    finally:
        p.terminate()
        assert p.wait(10) == 0


def test_a_restarted_broker_grows_back_when_old_tenants_exit(broker_exe, tmp_path):
    """After a broker restart, pods of the previous instance still hold their granules (imported
    dma-bufs keep the memory alive, measured on MI355X: docs/HBM_TURNOVER.md, exporter death).
    The new broker starts with what is free and takes the rest once it is back (the stub holds
    6 of 16 GiB for 1.5 s), zeroing the new granules before it lends them."""
    exe, libdir = broker_exe
    env = dict(os.environ, LD_LIBRARY_PATH=libdir, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1",
               FAKE_HIP_TOTAL_GIB="16", FAKE_HIP_HELD_GIB="6", FAKE_HIP_HELD_MS="1500")
    path = str(tmp_path / "hbm0.sock")
    p = subprocess.Popen([exe, "--socket", path, "--reserve-gib", "2", "--release-policy", "trust"],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
    try:
        ready = json.loads(p.stdout.readline())
        assert ready["granules"] == 8                       # 16 - 6 held - 2 reserve
        st = json.loads(_line(path + ".admin", "STAT"))
        assert st["granules_max"] == 14 and st["free"] == 8
        t = time.monotonic() + 10
        while time.monotonic() < t:
            st = json.loads(_line(path + ".admin", "STAT"))
            if st["granules"] == 14 and st["free"] == 14:
                break
            time.sleep(0.1)
        assert st["granules"] == 14 and st["grown"] == 6 and st["free"] == 14, st
        assert st["scrubbed_bytes"] >= 6 * GIB                # the new granules were zeroed first
        assert _line(path + ".admin", f"GRANT {'g' * 32} {13 * GIB}") == "OK 13"
        pod = Pod(path, "g" * 32)
        assert pod.result()[0] == f"FDS 13 {GIB}"
        pod.close()
    finally:
        p.terminate()
        assert p.wait(10) == 0


class Holder(StreamPod):
    """A pod's shim after its TAKE: asks for granules beyond its grant (EXTEND) and for what it
    could still borrow (AVAIL) on the same connection."""

    def ask(self, line, timeout=5.0):
        self.s.sendall(line.encode() + b"\n")
        return self.more(timeout)


def test_extend_lends_only_granules_no_grant_claims_up_to_the_limit(broker):
    """a pod may borrow granules beyond its grant, up to its quota (the
    grant's limit), but only granules no grant claims: a grant not taken yet is a pod about to
    start, and its granules must be there for it."""
    assert broker.admin(f"GRANT {'a' * 32} {4 * GIB} {7 * GIB + 5}") == "OK 4"   # limit: 7 whole granules
    assert broker.admin(f"GRANT {'b' * 32} {2 * GIB}") == "OK 2"                  # not taken yet
    a = Holder(broker.path, "a" * 32)
    assert a.result()[0] == f"FDS 4 {GIB} 4 7"
    assert broker.stat()["uncommitted"] == 2
    assert a.ask("AVAIL")[0] == "AVAIL 2"
    head, fds = a.ask("EXTEND 5")
    assert head == f"XFDS 2 {GIB}" and len(fds) == 2
    assert a.ask("AVAIL")[0] == "AVAIL 0" and a.ask("EXTEND 1")[0] == f"XFDS 0 {GIB}"
    b = Pod(broker.path, "b" * 32)
    assert b.result()[0] == f"FDS 2 {GIB}"                   # the grant's granules were kept for it
    st = broker.stat()
    assert st["extra"] == 2 and st["extended"] == 2 and st["extends"] == 2 and st["held"] == 8 and st["free"] == 0
    a.close()                                                # borrowed granules return with the rest
    time.sleep(0.3)
    st = broker.stat()
    assert st["extra"] == 0 and st["free"] == 6 and st["held"] == 2
    b.close()


def test_extend_respects_the_limit_and_a_revoked_holder_gets_nothing(broker):
    assert broker.admin(f"GRANT {'c' * 32} {2 * GIB} {3 * GIB}") == "OK 2"
    c = Holder(broker.path, "c" * 32)
    assert c.result()[0] == f"FDS 2 {GIB} 2 3"
    assert c.ask("EXTEND 4")[0] == f"XFDS 1 {GIB}"           # 3 granules at most
    assert c.ask("EXTEND 1")[0] == f"XFDS 0 {GIB}"
    assert broker.admin(f"REVOKE {'c' * 32}") == "OK 3"
    assert c.more()[0] == "END"
    assert c.ask("EXTEND 1")[0] == f"XFDS 0 {GIB}" and c.ask("AVAIL")[0] == "AVAIL 0"
    c.close()


def test_owed_granules_that_never_come_are_cancelled_and_the_next_taker_is_answered(broker_exe, tmp_path):
    """a streaming taker owed granules that never come back (a holder that keeps them)
    must not hold up the takers behind it for ever: at --wait-s its stream is ended ("END": the
    shim shrinks its grant to what it has and uses the driver for the rest), and the next taker
    is served or ended in its turn."""
    b = Broker(broker_exe, str(tmp_path / "hbm0.sock"), wait_s=1.0)
    try:
        b.admin(f"GRANT {'h' * 32} {6 * GIB}")
        b.admin(f"GRANT {'s' * 32} {4 * GIB}")
        b.admin(f"GRANT {'q' * 32} {1 * GIB}")
        holder = Pod(b.path, "h" * 32)
        assert holder.result()[0] == f"FDS 6 {GIB}"
        t0 = time.monotonic()
        s = StreamPod(b.path, "s" * 32)
        assert s.result()[0] == f"FDS 2 {GIB} 4 4"
        q = StreamPod(b.path, "q" * 32)
        assert q.result()[0] == f"FDS 0 {GIB} 1 1"
        assert s.more(timeout=3)[0] == "END" and 0.9 < time.monotonic() - t0 < 2.5
        assert q.more(timeout=3)[0] == "END" and time.monotonic() - t0 < 3.5
        st = b.stat()
        assert st["ends"] == 2 and st["owed"] == 0 and st["held"] == 8
        for p in (holder, s, q):
            p.close()
    finally:
        b.stop()


def test_size_gives_granules_back_and_takes_them_again(broker_exe, tmp_path):
    """SIZE sets how much of the GPU the broker may hold (the plugin sends
    SIZE 0 on a cgpu.disable.isolation node). Free granules go back to the driver at once, lent
    ones when they come back; SIZE max grows it again."""
    b = Broker(broker_exe, str(tmp_path / "hbm0.sock"))
    try:
        b.admin(f"GRANT {'a' * 32} {2 * GIB}")
        a = Pod(b.path, "a" * 32)
        assert a.result()[0] == f"FDS 2 {GIB}"
        assert b.admin("SIZE 0") == "OK 2 0"                 # the 2 lent granules cannot go yet
        st = b.stat()
        assert st["granules"] == 2 and st["target"] == 0 and st["given_back"] == 6 and st["free"] == 0
        a.close()
        deadline = time.time() + 5
        while b.stat()["granules"] and time.time() < deadline:
            time.sleep(0.05)
        assert b.stat()["granules"] == 0
        assert b.admin("SIZE max") == "OK 8 8"               # taken again at once
        deadline = time.time() + 5
        while b.stat()["free"] < 8 and time.time() < deadline:
            time.sleep(0.05)
        st = b.stat()
        assert st["free"] == 8 and st["scrubbed_bytes"] >= 10 * GIB   # new granules are zeroed first
        assert b.admin("SIZE 3") == "OK 3 3" and b.stat()["free"] == 3
        assert b.admin("SIZE -1").startswith("ERR") and b.admin("SIZE 99") == "OK 8 8"   # capped at its size
    finally:
        b.stop()


def test_start_empty_holds_nothing_until_sized(broker_exe, tmp_path):
    """--start-empty (the DaemonSet): nothing is held until the granter says how much, and the
    release policy is still chosen from the kernel (a throwaway export: here the stub's memfds,
    which fdinfo does not count, so "exit"); an explicit "refs" on such a kernel refuses to run
    (the choice no longer depends on a granule 0 that may not exist)."""
    b = Broker(broker_exe, str(tmp_path / "hbm0.sock"), policy="auto", extra=("--start-empty",))
    try:
        assert b.ready["granules"] == 0 and b.ready["release_policy"] == "exit"
        assert b.stat()["target"] == 0
        assert b.admin("SIZE max") == "OK 8 8"
    finally:
        b.stop()
    exe, libdir = broker_exe
    r = subprocess.run([exe, "--socket", str(tmp_path / "x.sock"), "--gib", "4", "--release-policy", "refs",
                        "--start-empty"], env=dict(os.environ, LD_LIBRARY_PATH=libdir, ASAN_OPTIONS="detect_leaks=0"),
                       capture_output=True, text=True, timeout=30)
    assert r.returncode == 2 and "needs the dma-buf count" in r.stderr


def test_driver_pressure_gives_free_granules_back_and_the_broker_grows_again(broker_exe, tmp_path):
    """when the driver runs short (here "another process" takes 3 of the 4 GiB
    the broker left it, for 1.5 s), free granules no grant claims go back to the driver until it
    has --low-water-gib free; once it has more than the reserve again the broker grows back."""
    b = Broker(broker_exe, str(tmp_path / "hbm0.sock"), gib=12, extra=("--low-water-gib", "3"),
               env={"FAKE_HIP_TOTAL_GIB": "16", "FAKE_HIP_LATE_GIB": "3", "FAKE_HIP_LATE_MS": "600",
                    "FAKE_HIP_LATE_FOR_MS": "1500"})
    try:
        b.admin(f"GRANT {'g' * 32} {4 * GIB}")
        deadline = time.time() + 5
        st = b.stat()
        while st["pressure_given"] < 2 and time.time() < deadline:
            time.sleep(0.05)
            st = b.stat()
        assert st["pressure_given"] == 2 and st["granules"] == 10, st   # driver: 1 -> 3 GiB free
        deadline = time.time() + 8
        while st["granules"] < 12 and time.time() < deadline:
            time.sleep(0.1)
            st = b.stat()
        assert st["granules"] == 12 and st["grown"] >= 2, st
        p = Pod(b.path, "g" * 32)                                        # the grant was never short
        assert p.result()[0] == f"FDS 4 {GIB}"
        p.close()
    finally:
        b.stop()
