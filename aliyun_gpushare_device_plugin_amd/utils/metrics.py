"""Metrics: Allocate phase spans, outcomes, device health — Prometheus text exposition.

The reference has no metrics at all; this is the new build's observability
layer. Kept dependency-free (a registry per plugin instance, so tests do not fight over a
process-global registry); ``serve()`` exposes ``/metrics`` and ``/healthz``.
"""
from __future__ import annotations

import bisect
import http.server
import threading
import time
from contextlib import contextmanager

_DEFAULT_BUCKETS = (0.0001, 0.00025, 0.0005, 0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1,
                    0.25, 0.5, 1.0, 2.5, 5.0, 10.0)


def _labels_key(labels: dict) -> tuple:
    return tuple(sorted(labels.items()))


def _fmt_labels(key: tuple) -> str:
    if not key:
        return ""
    return "{" + ",".join(f'{k}="{v}"' for k, v in key) + "}"


class Counter:
    def __init__(self, name: str, help_: str):
        self.name, self.help = name, help_
        self._v: dict[tuple, float] = {}
        self._lock = threading.Lock()

    def inc(self, amount: float = 1.0, **labels):
        k = _labels_key(labels)
        with self._lock:
            self._v[k] = self._v.get(k, 0.0) + amount

    def value(self, **labels) -> float:
        return self._v.get(_labels_key(labels), 0.0)

    def render(self):
        yield f"# HELP {self.name} {self.help}\n# TYPE {self.name} counter\n"
        for k, v in sorted(self._v.items()):
            yield f"{self.name}{_fmt_labels(k)} {v}\n"


class Gauge(Counter):
    def set(self, value: float, **labels):
        with self._lock:
            self._v[_labels_key(labels)] = float(value)

    def clear(self):
        with self._lock:
            self._v.clear()

    def render(self):
        yield f"# HELP {self.name} {self.help}\n# TYPE {self.name} gauge\n"
        for k, v in sorted(self._v.items()):
            yield f"{self.name}{_fmt_labels(k)} {v}\n"


class Histogram:
    """Cumulative-bucket histogram plus a bounded reservoir for exact quantiles."""

    def __init__(self, name: str, help_: str, buckets=_DEFAULT_BUCKETS, reservoir: int = 100_000):
        self.name, self.help, self.buckets = name, help_, tuple(buckets)
        self._counts: dict[tuple, list] = {}
        self._sum: dict[tuple, float] = {}
        self._samples: dict[tuple, list] = {}
        self._reservoir = reservoir
        self._lock = threading.Lock()

    def observe(self, value: float, **labels):
        k = _labels_key(labels)
        with self._lock:
            c = self._counts.setdefault(k, [0] * (len(self.buckets) + 1))
            c[bisect.bisect_left(self.buckets, value)] += 1
            self._sum[k] = self._sum.get(k, 0.0) + value
            s = self._samples.setdefault(k, [])
            if len(s) < self._reservoir:
                s.append(value)

    @contextmanager
    def time(self, **labels):
        t0 = time.perf_counter()
        try:
            yield
        finally:
            self.observe(time.perf_counter() - t0, **labels)

    def samples(self, **labels) -> list:
        return list(self._samples.get(_labels_key(labels), []))

    def quantile(self, q: float, **labels) -> float | None:
        s = sorted(self._samples.get(_labels_key(labels), []))
        if not s:
            return None
        idx = min(len(s) - 1, max(0, int(round(q * (len(s) - 1)))))
        return s[idx]

    def count(self, **labels) -> int:
        return sum(self._counts.get(_labels_key(labels), []))

    def summary(self, qs=(0.5, 0.9, 0.99)) -> list[dict]:
        """Exact quantiles from the reservoir, one entry per label set."""
        with self._lock:
            items = [(k, sorted(v)) for k, v in self._samples.items()]
        out = []
        for k, s in items:
            if not s:
                continue
            d = {"labels": dict(k), "count": len(s)}
            for q in qs:
                d[f"p{int(q * 100)}"] = s[min(len(s) - 1, max(0, int(round(q * (len(s) - 1)))))]
            out.append(d)
        return out

    def reset(self):
        with self._lock:
            self._counts.clear()
            self._sum.clear()
            self._samples.clear()

    def render(self):
        yield f"# HELP {self.name} {self.help}\n# TYPE {self.name} histogram\n"
        for k, counts in sorted(self._counts.items()):
            acc = 0
            for b, c in zip(self.buckets, counts):
                acc += c
                lk = _fmt_labels(k + (("le", repr(b)),))
                yield f"{self.name}_bucket{lk} {acc}\n"
            acc += counts[-1]
            yield f"{self.name}_bucket{_fmt_labels(k + (('le', '+Inf'),))} {acc}\n"
            yield f"{self.name}_sum{_fmt_labels(k)} {self._sum.get(k, 0.0)}\n"
            yield f"{self.name}_count{_fmt_labels(k)} {acc}\n"


class Registry:
    def __init__(self):
        self._m: dict[str, object] = {}
        self._lock = threading.Lock()
        self._collectors: list = []     # fn() -> exposition text, read at scrape time

    def _get(self, cls, name, help_, **kw):
        with self._lock:
            if name not in self._m:
                self._m[name] = cls(name, help_, **kw)
            return self._m[name]

    def counter(self, name, help_=""):
        return self._get(Counter, name, help_)

    def histograms(self) -> dict:
        with self._lock:
            return {n: m for n, m in self._m.items() if isinstance(m, Histogram)}

    def gauge(self, name, help_=""):
        return self._get(Gauge, name, help_)

    def histogram(self, name, help_="", **kw):
        return self._get(Histogram, name, help_, **kw)

    def add_collector(self, fn) -> None:
        self._collectors.append(fn)

    def render(self) -> str:
        out = []
        for m in list(self._m.values()):
            out.extend(m.render())
        for fn in list(self._collectors):
            try:
                out.append(fn())
            except Exception:  # noqa: BLE001 - a collector never fails the scrape
                pass
        return "".join(out)


def native_server_exposition(st: dict) -> str:
    """The native DevicePlugin server's counters (``gs_dp_stats``) as Prometheus text."""
    if not st:
        return ""
    lines = [
        "# HELP gpushare_native_allocate_total Allocates the native server answered from the prepared table "
        "(native) or handed to the engine (forwarded)\n# TYPE gpushare_native_allocate_total counter\n",
        f'gpushare_native_allocate_total{{path="native"}} {st.get("fast", 0)}\n',
        f'gpushare_native_allocate_total{{path="forwarded"}} {st.get("forwarded_allocate", 0)}\n',
        "# HELP gpushare_native_declined_total Why an Allocate was left to the engine\n"
        "# TYPE gpushare_native_declined_total counter\n"]
    lines += [f'gpushare_native_declined_total{{reason="{k}"}} {v}\n'
              for k, v in sorted((st.get("declined") or {}).items())]
    for name, key, kind, help_ in (
            ("gpushare_native_forwarded_requests_total", "forwarded", "counter", "Requests handed to Python handlers"),
            ("gpushare_native_table_waits_total", "waited", "counter",
             "Allocates that waited for the table to catch up with the pod cache"),
            ("gpushare_native_connections_total", "connections", "counter", "Kubelet connections accepted"),
            ("gpushare_native_listandwatch_sends_total", "law_sends", "counter", "ListAndWatch messages sent"),
            ("gpushare_native_journal_used_bytes", "journal_used", "gauge", "Bytes in the native answers' journal"),
            ("gpushare_native_claims_pending", "taken_pending", "gauge",
             "Native answers not yet taken in by the engine's bookkeeping")):
        lines.append(f"# HELP {name} {help_}\n# TYPE {name} {kind}\n{name} {st.get(key, 0)}\n")
    return "".join(lines)


class PluginMetrics:
    """The plugin's metric set."""

    def __init__(self, registry: Registry | None = None):
        r = self.registry = registry or Registry()
        self.allocate_latency = r.histogram("gpushare_allocate_latency_seconds",
                                            "Allocate RPC latency by phase (prelude/lock/lookup/decide/patch/total)")
        self.allocate_outcomes = r.counter("gpushare_allocate_total", "Allocate outcomes")
        self.table_publish = r.histogram("gpushare_native_table_publish_seconds",
                                         "Time to build and publish the native Allocate table: from the pod-cache "
                                         "hook (one pod changed) or the prepare loop (full rebuild)")
        self.table_publish_skipped = r.counter("gpushare_native_table_hook_skipped_total",
                                               "Pod-cache changes the hook left to the prepare loop (its last table "
                                               "was not at the previous version / engine generation)")
        self.allocate_requests = r.histogram("gpushare_allocate_apiserver_requests",
                                             "apiserver requests made on the Allocate path (counted by the handler "
                                             "thread; write-behind patches excluded)", buckets=(0, 1, 2, 3, 4, 8))
        self.pending_match_failures = r.counter("gpushare_pending_match_failures_total",
                                                "Allocates with no matching assumed pod")
        self.units_per_gpu = r.gauge("gpushare_advertised_units", "Advertised gpu-mem units per GPU")
        self.unit_fallback = r.gauge("gpushare_memory_unit_fallback",
                                     "1 if --memory-unit=MiB was replaced by GiB (fake-device limit)")
        self.health_events_armed = r.gauge("gpushare_health_events_armed",
                                           "GPUs with SMI event notification (reset / VM fault) armed")
        self.health_ecc_readable = r.gauge("gpushare_health_ecc_readable", "GPUs whose ECC counters were read")
        self.health_degraded = r.gauge("gpushare_health_degraded",
                                       "1 if SMI event notification is not armed on every GPU (alert: /dev/kfd "
                                       "not accessible; resets seen by polling only)")
        self.config_error = r.gauge("gpushare_config_error", "1 if the plugin parked on an impossible config")
        self.device_health = r.gauge("gpushare_device_healthy", "1 if the GPU is healthy")
        self.hbm_used = r.gauge("gpushare_hbm_used_bytes", "HBM in use per GPU (SMI)")
        self.cache_events = r.counter("gpushare_pod_cache_events_total", "Pod watch-cache events")
        self.listandwatch_sends = r.counter("gpushare_listandwatch_sends_total", "Device list sends")
        # quota shim ledgers (--ledger-dir): what each shared container actually holds
        self.shim_used = r.gauge("gpushare_container_hbm_used_bytes", "HBM held by a container (shim ledger)")
        self.shim_quota = r.gauge("gpushare_container_hbm_quota_bytes", "Container HBM quota (shim ledger)")
        self.shim_peak = r.gauge("gpushare_container_hbm_peak_bytes", "Container HBM high-water mark (shim ledger)")
        self.shim_denied = r.gauge("gpushare_container_quota_denials", "Allocations refused by the quota shim")
        # quota watchdog (quota/watchdog.py): kernel-reported HBM per pod vs its share
        self.quota_violation = r.gauge("gpushare_quota_violation_bytes",
                                       "HBM a pod holds on a GPU beyond its share (DRM fdinfo), per pod and GPU")
        self.pod_hbm_used = r.gauge("gpushare_pod_hbm_used_bytes",
                                    "HBM a pod's processes hold on a GPU (kernel-reported, DRM fdinfo)")
        self.quota_violations_total = r.counter("gpushare_quota_violations_total", "Quota violations detected")
        self.quota_kills = r.counter("gpushare_quota_kills_total", "Processes killed by the quota watchdog")
        self.unaccounted_hbm = r.gauge("gpushare_unaccounted_hbm_bytes",
                                       "HBM held on a GPU by processes of no pod on this node")
        self.enforcement_mode = r.gauge("gpushare_enforcement_mode",
                                        "1 on the effective HBM-share enforcement for tenants without the shim: "
                                        "dmem (kernel limit), kill (watchdog), report or off")
        self.dmem_limited_pods = r.gauge("gpushare_dmem_limited_pods",
                                         "Shared pods whose HBM share is a kernel dmem.max limit on their cgroup")
        self.cu_slots_held = r.gauge("gpushare_cu_slots_held",
                                     "CU slots held by pods per GPU at the last compute-isolation decision "
                                     "(slot = one CU on every XCD; > slots per GPU means oversubscribed)")


def serve(registry: Registry, addr: str, health_fn=None, ready_fn=None,
          debug_fn=None) -> http.server.ThreadingHTTPServer:
    """Start ``/metrics`` + ``/healthz`` + ``/readyz`` + ``/debug/latency`` on ``host:port`` in a
    daemon thread. ``ready_fn() -> (ok, reason)`` backs ``/readyz`` (503 + reason when not ready).

    ``/debug/latency`` returns exact p50/p90/p99 of every histogram (JSON), plus whatever
    ``debug_fn()`` returns (the native server's counters); ``?reset=1`` also clears the
    histograms, honoured only with ``GPUSHARE_DEBUG=1`` (benchmarks bracket a timed region)."""
    import json as _json
    import os as _os

    host, _, port = addr.rpartition(":")

    class H(http.server.BaseHTTPRequestHandler):
        def do_GET(self):
            if self.path.startswith("/metrics"):
                body, ctype, code = registry.render().encode(), "text/plain; version=0.0.4", 200
            elif self.path.startswith("/debug/latency"):
                hs = registry.histograms()
                d = {n: h.summary() for n, h in hs.items()}
                if debug_fn is not None:
                    try:
                        d.update(debug_fn())
                    except Exception:  # noqa: BLE001 - a debug view never fails the endpoint
                        pass
                body = _json.dumps(d).encode()
                ctype, code = "application/json", 200
                if "reset=1" in self.path and _os.environ.get("GPUSHARE_DEBUG") == "1":
                    for h in hs.values():
                        h.reset()
            elif self.path.startswith("/readyz"):
                ok, why = (True, "ok") if ready_fn is None else ready_fn()
                body, ctype, code = why.encode(), "text/plain", 200 if ok else 503
            elif self.path.startswith("/healthz"):
                ok = True if health_fn is None else bool(health_fn())
                body, ctype, code = (b"ok" if ok else b"unhealthy"), "text/plain", 200 if ok else 503
            else:
                body, ctype, code = b"not found", "text/plain", 404
            self.send_response(code)
            self.send_header("Content-Type", ctype)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def log_message(self, *a):
            pass

    srv = http.server.ThreadingHTTPServer((host or "0.0.0.0", int(port)), H)
    srv.daemon_threads = True
    threading.Thread(target=srv.serve_forever, name="metrics", daemon=True).start()
    return srv
