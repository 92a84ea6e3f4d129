"""HTTP server over real sockets: status codes, keep-alive, pipelining, gzip, HEAD,
readiness, and snapshot consistency under concurrent scraping at 100 Hz sampling."""
import gzip
import http.client
import socket
import threading
import time

import pytest

from kubernetes_gpu_exporter_amd.utils import promtext


def req(port, path, method="GET", headers=None):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=5)
    c.request(method, path, headers=headers or {})
    r = c.getresponse()
    body = r.read()
    c.close()
    return r, body


def test_not_ready_before_first_tick(mock_engine):
    e = mock_engine(1)
    r, body = req(e.http_port, "/metrics")
    assert r.status == 503
    r, _ = req(e.http_port, "/readyz")
    assert r.status == 503
    r, body = req(e.http_port, "/healthz")
    assert r.status == 200 and body == b"ok\n"


def test_metrics_endpoint(mock_engine):
    e = mock_engine(1)
    e.tick(1_000_000_000)
    r, body = req(e.http_port, "/metrics")
    assert r.status == 200
    assert r.getheader("Content-Type") == "text/plain; version=0.0.4; charset=utf-8"
    assert body.decode() == e.snapshot_text()
    promtext.parse(body.decode())
    r, body = req(e.http_port, "/metrics?x=1")
    assert r.status == 200
    r, _ = req(e.http_port, "/readyz")
    assert r.status == 200
    r, body = req(e.http_port, "/metrics", method="HEAD")
    assert r.status == 200 and body == b"" and int(r.getheader("Content-Length")) > 0
    r, _ = req(e.http_port, "/nope")
    assert r.status == 404
    r, _ = req(e.http_port, "/metrics", method="POST")
    assert r.status == 405
    r, body = req(e.http_port, "/")
    assert r.status == 200 and b"/metrics" in body


def test_custom_path(mock_engine, native):
    c = native.HttpConfig()
    e = mock_engine(1)
    e.tick(1)
    # default path; a custom path is exercised through the exporter config test
    r, _ = req(e.http_port, "/metrics")
    assert r.status == 200


def test_keepalive_and_pipelining(mock_engine):
    e = mock_engine(1)
    e.tick(1_000_000_000)
    s = socket.create_connection(("127.0.0.1", e.http_port))
    s.sendall(b"GET /metrics HTTP/1.1\r\nHost: x\r\n\r\nGET /healthz HTTP/1.1\r\nHost: x\r\n\r\n"
              b"GET /metrics HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n")
    data = b""
    while True:
        chunk = s.recv(1 << 16)
        if not chunk:
            break
        data += chunk
    s.close()
    assert data.count(b"HTTP/1.1 200 OK") == 3
    assert b"Connection: close" in data


def test_pipelined_request_behind_a_partial_write(native):
    """A response too big for the socket buffer completes on the EPOLLOUT path; the
    request pipelined behind it (already read) must be answered then, not at idle timeout."""
    c = native.EngineConfig()
    c.backend = "mock"
    c.mock_devices = 8
    c.series_profile = "full"
    c.interval_s = 0
    c.http.host = "127.0.0.1"
    c.http.port = 0
    c.http.socket_sndbuf = 4096
    e = native.Engine(c)
    e.start()
    try:
        e.tick(1_000_000_000)
        body_len = len(e.snapshot_text())
        assert body_len > 32 << 10
        s = socket.socket()
        s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4096)  # before connect: small window
        s.connect(("127.0.0.1", e.http_port))
        s.sendall(b"GET /metrics HTTP/1.1\r\nHost: x\r\n\r\nGET /healthz HTTP/1.1\r\nHost: x\r\n\r\n")
        time.sleep(0.3)  # let the server fill both buffers and park on EPOLLOUT
        s.settimeout(3.0)
        data = b""
        t0 = time.monotonic()
        while not data.endswith(b"ok\n"):
            chunk = s.recv(1 << 16)
            assert chunk, "connection closed early"
            data += chunk
        assert time.monotonic() - t0 < 3.0
        assert data.count(b"HTTP/1.1 200 OK") == 2
        s.close()
    finally:
        e.stop()


def test_gzip_negotiation(mock_engine):
    e = mock_engine(1)
    e.tick(1_000_000_000)
    r, body = req(e.http_port, "/metrics", headers={"Accept-Encoding": "gzip"})
    # the snapshot has no gzip copy yet: the worker compresses this response itself
    assert r.status == 200 and r.getheader("Content-Encoding") == "gzip"
    assert gzip.decompress(body).decode() == e.snapshot_text()
    assert e.stats()["http_gzip_on_demand"] == 1
    e.tick(1_100_000_000)  # unsteady gzip client: the sampler pre-compresses each tick
    assert e.stats()["gzip_eager"] == 1
    r, body = req(e.http_port, "/metrics", headers={"Accept-Encoding": "gzip, deflate"})
    assert r.getheader("Content-Encoding") == "gzip"
    assert gzip.decompress(body).decode() == e.snapshot_text()
    assert e.stats()["http_gzip_on_demand"] == 1
    r, body = req(e.http_port, "/metrics")
    assert r.getheader("Content-Encoding") is None


def test_bad_request_closes(mock_engine):
    e = mock_engine(1)
    s = socket.create_connection(("127.0.0.1", e.http_port))
    s.sendall(b"GARBAGE\r\n\r\n")
    data = s.recv(4096)
    assert b"400" in data
    s.close()


def _closed(s, timeout):
    s.settimeout(timeout)
    try:
        return s.recv(4096) == b""
    except ConnectionResetError:
        return True


def test_oversized_header_closes(mock_engine):
    """A request head that never ends is cut off at 16 KiB: no unbounded buffering."""
    e = mock_engine(1)
    e.tick(1)
    s = socket.create_connection(("127.0.0.1", e.http_port))
    s.sendall(b"GET /metrics HTTP/1.1\r\n" + b"X-Filler: " + b"a" * 20000)
    assert _closed(s, 3)
    s.close()
    r, _ = req(e.http_port, "/healthz")  # the server itself is fine
    assert r.status == 200


def test_idle_and_slow_clients_are_swept(native):
    """A connection that stops mid-request (slowloris) or idles is closed after
    idle_timeout_ms; a live keep-alive client on the same worker is unaffected."""
    c = native.EngineConfig()
    c.backend = "mock"
    c.interval_s = 0
    c.http.host = "127.0.0.1"
    c.http.port = 0
    c.http.idle_timeout_ms = 1000
    e = native.Engine(c)
    e.start()
    try:
        e.tick(1)
        slow = socket.create_connection(("127.0.0.1", e.http_port))
        slow.sendall(b"GET /metrics HTTP/1.1\r\nHost: x\r\n")  # never finished
        idle = socket.create_connection(("127.0.0.1", e.http_port))
        t0 = time.monotonic()
        assert _closed(slow, 5) and _closed(idle, 5)
        assert 0.9 < time.monotonic() - t0 < 4.0
        r, _ = req(e.http_port, "/healthz")
        assert r.status == 200
    finally:
        e.stop()


def test_concurrent_scrapes_see_consistent_snapshots(native):
    """Sampler at 100 Hz + 4 scraper threads: every body parses and ticks never go back."""
    c = native.EngineConfig()
    c.backend = "mock"
    c.mock_devices = 8
    c.interval_s = 0.01
    c.http.host = "127.0.0.1"
    c.http.port = 0
    c.http.threads = 2
    e = native.Engine(c)
    e.start()
    try:
        deadline = time.time() + 5
        while time.time() < deadline:
            r, _ = req(e.http_port, "/readyz")
            if r.status == 200:
                break
            time.sleep(0.01)
        errors = []

        def scraper():
            conn = http.client.HTTPConnection("127.0.0.1", e.http_port, timeout=5)
            last = -1
            for _ in range(60):
                conn.request("GET", "/metrics")
                body = conn.getresponse().read().decode()
                try:
                    fams = promtext.parse(body)
                    t = promtext.value(fams, "gpuexp_ticks_total")
                    if t < last:
                        errors.append(f"ticks went back {last}->{t}")
                    last = t
                    # one consistent tick: all 8 GPUs present in every family we check
                    assert len(fams["amd_gpu_up"].samples) == 8
                except Exception as ex:  # noqa: BLE001
                    errors.append(repr(ex))
            conn.close()

        th = [threading.Thread(target=scraper) for _ in range(4)]
        [t.start() for t in th]
        [t.join() for t in th]
        assert not errors, errors[:3]
    finally:
        e.stop()


def test_native_scrape_client(mock_engine, native):
    e = mock_engine(2)
    e.tick(1_000_000_000)
    r = native.scrape_loop("127.0.0.1", e.http_port, "/metrics", hz=0, count=50, keep_last_body=True)
    assert r["errors"] == 0 and r["non200"] == 0 and len(r["latency_ns"]) == 50
    assert r["last_body"].decode() == e.snapshot_text()
    r = native.scrape_loop("127.0.0.1", e.http_port, "/metrics", hz=200, count=20, keepalive=False)
    assert r["errors"] == 0 and 0.08 < r["wall_s"] < 1.0


def test_many_connections(mock_engine):
    e = mock_engine(1)
    e.tick(1)
    socks = [socket.create_connection(("127.0.0.1", e.http_port)) for _ in range(200)]
    for s in socks:
        s.sendall(b"GET /healthz HTTP/1.1\r\nHost: x\r\n\r\n")
    for s in socks:
        assert s.recv(4096).startswith(b"HTTP/1.1 200")
        s.close()
    assert e.stats()["http_requests"] >= 200


PB_CT = "application/vnd.google.protobuf; proto=io.prometheus.client.MetricFamily; encoding=delimited"


def test_protobuf_negotiation_matches_text(mock_engine):
    """A Prometheus-style Accept header gets the delimited MetricFamily protobuf (from the
    tick after the first ask), with exactly the text exposition's families and values."""
    import math
    from kubernetes_gpu_exporter_amd.utils import promproto
    e = mock_engine(2, enable_counters=True, enable_sentinel=True)
    e.tick(1_000_000_000)
    r, body = req(e.http_port, "/metrics", headers={"Accept": promproto.ACCEPT})
    assert r.status == 200  # first ask: text until the sampler renders protobuf
    e.tick(2_000_000_000)
    r, pb = req(e.http_port, "/metrics", headers={"Accept": promproto.ACCEPT})
    assert r.getheader("Content-Type") == PB_CT
    _, text = req(e.http_port, "/metrics")
    fams_txt = promtext.parse(text.decode())
    fams_pb = promproto.to_samples(promproto.parse_delimited(pb))
    assert list(fams_pb) == sorted(fams_pb) == sorted(fams_txt)
    for name, (typ, helptext, rows) in fams_pb.items():
        ft = fams_txt[name]
        assert ft.type == typ and ft.help == helptext, name
        want = sorted((s, tuple(sorted((k, v) for k, v in lab.items() if k != "le")),
                       float(lab["le"]) if "le" in lab else None, v) for s, lab, v in ft.samples)
        got = sorted((s, tuple(sorted((k, v) for k, v in lab.items() if k != "le")),
                      lab.get("le"), v) for s, lab, v in rows)
        assert len(want) == len(got), name
        for w, g in zip(want, got):
            assert w[:3] == g[:3], (name, w, g)
            assert (math.isnan(w[3]) and math.isnan(g[3])) or abs(w[3] - g[3]) <= 1e-9 * max(1.0, abs(w[3])), (w, g)
    # gzip on top of protobuf
    r, z = req(e.http_port, "/metrics", headers={"Accept": promproto.ACCEPT, "Accept-Encoding": "gzip"})
    e.tick(3_000_000_000)
    r, z = req(e.http_port, "/metrics", headers={"Accept": promproto.ACCEPT, "Accept-Encoding": "gzip"})
    assert r.getheader("Content-Encoding") == "gzip" and r.getheader("Content-Type") == PB_CT
    assert promproto.parse_delimited(gzip.decompress(z))


@pytest.mark.parametrize("accept,proto", [
    ("text/plain;version=0.0.4;q=0.9,application/vnd.google.protobuf;proto=io.prometheus.client.MetricFamily;"
     "encoding=delimited;q=0.5", False),
    ("application/vnd.google.protobuf;proto=io.prometheus.client.MetricFamily;encoding=text", False),
    ("application/openmetrics-text;version=1.0.0,text/plain;version=0.0.4;q=0.5", False),
    ("*/*", False),
    ("application/vnd.google.protobuf;proto=io.prometheus.client.MetricFamily;encoding=delimited", True),
])
def test_protobuf_negotiation_respects_q(mock_engine, accept, proto):
    e = mock_engine(1)
    e.tick(1_000_000_000)
    req(e.http_port, "/metrics", headers={"Accept": accept})
    e.tick(2_000_000_000)
    r, _ = req(e.http_port, "/metrics", headers={"Accept": accept})
    assert (r.getheader("Content-Type") == PB_CT) is proto


def test_scrape_timing_split(mock_engine, native):
    """X-Gpuexp-Timing: the server echoes (request parsed, write started) on the client's
    clock (same host, CLOCK_MONOTONIC), so the bench can split a scrape's latency; the
    body is unchanged and a request without the header gets no timing header."""
    e = mock_engine(1)
    e.tick(1_000_000_000)
    c = native.ScrapeClient("127.0.0.1", e.http_port, "/metrics", timing=True)
    for _ in range(5):
        assert c.scrape() > 0
        t_send, t_parse, t_write, t_done = c.last_timing()
        assert 0 < t_send <= t_parse <= t_write <= t_done
    assert c.last_body().decode() == e.snapshot_text()
    plain = native.ScrapeClient("127.0.0.1", e.http_port, "/metrics")
    assert plain.scrape() > 0 and plain.last_timing()[1] == 0
    s = socket.create_connection(("127.0.0.1", e.http_port))
    s.sendall(b"GET /metrics HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n")
    head = b""
    while b"\r\n\r\n" not in head:
        head += s.recv(65536)
    s.close()
    assert b"X-Gpuexp-Timing" not in head.split(b"\r\n\r\n")[0]


def test_listen_all_interfaces_is_dual_stack(native):
    """":8000" (empty host) listens like Go's ListenAndServe(":8000") (main.go:71): IPv4
    and IPv6 clients both reach it; an explicit IPv4 host stays IPv4-only."""
    c = native.EngineConfig()
    c.backend = "mock"
    c.interval_s = 0
    c.http.host = ""
    c.http.port = 0
    e = native.Engine(c)
    e.start()
    try:
        e.tick(1_000_000_000)
        port = e.http_port
        for fam, addr in ((socket.AF_INET, "127.0.0.1"), (socket.AF_INET6, "::1")):
            try:
                s = socket.socket(fam, socket.SOCK_STREAM)
                s.settimeout(5)
                s.connect((addr, port))
            except OSError as ex:
                if fam == socket.AF_INET6:
                    pytest.skip(f"no IPv6 loopback here: {ex}")
                raise
            s.sendall(b"GET /healthz HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n")
            assert s.recv(4096).startswith(b"HTTP/1.1 200"), fam
            s.close()
    finally:
        e.stop()


def test_readyz_reports_a_stalled_sampler(native):
    """A sampler stuck in a driver call keeps the last snapshot on /metrics (whose
    gpuexp_last_sample_timestamp_seconds then ages) while /readyz turns 503 once the
    snapshot is older than stale_after, and recovers with the next tick."""
    c = native.EngineConfig()
    c.backend = "mock"
    c.interval_s = 0
    c.http.host = "127.0.0.1"
    c.http.port = 0
    c.http.stale_after_ns = 300_000_000
    e = native.Engine(c)
    e.start()
    try:
        def get(path):
            conn = http.client.HTTPConnection("127.0.0.1", e.http_port, timeout=5)
            conn.request("GET", path)
            r = conn.getresponse()
            out = r.status, r.read().decode()
            conn.close()
            return out
        assert get("/readyz")[0] == 503  # no sample yet
        e.tick(1_000_000_000)
        assert get("/readyz")[0] == 200
        ts = promtext.value(promtext.parse(get("/metrics")[1]), "gpuexp_last_sample_timestamp_seconds")
        assert abs(ts - time.time()) < 5
        time.sleep(0.5)
        st, body = get("/readyz")
        assert st == 503 and body.startswith("stale: last sample"), body
        assert get("/metrics")[0] == 200  # still served: last known values beat none
        e.tick(2_000_000_000)
        assert get("/readyz")[0] == 200
    finally:
        e.stop()


def test_scrape_prewake_learns_a_steady_period(native):
    """A scraper with a steady period (here 30 ms) is learnt after 2 intervals: the worker
    then wakes on a timer just ahead of each expected request (short sleeps keep its core
    out of deep idle) — a few timer wake-ups per scrape, none once scraping stops, and none
    with prewake off."""
    def run(prewake: bool):
        c = native.EngineConfig()
        c.backend = "mock"
        c.interval_s = 0
        c.http.host = "127.0.0.1"
        c.http.port = 0
        c.http.prewake = prewake
        e = native.Engine(c)
        e.start()
        try:
            e.tick(1_000_000_000)
            cl = native.ScrapeClient("127.0.0.1", e.http_port, "/metrics")
            t = time.monotonic()
            for _ in range(14):
                t += 0.030
                time.sleep(max(0.0, t - time.monotonic()))
                assert cl.scrape() > 0
            woke = e.stats()["http_prewake_timer_wakeups"]
            time.sleep(0.2)  # scraper gone: the window closes, the timer stays disarmed
            later = e.stats()["http_prewake_timer_wakeups"]
            return woke, later
        finally:
            e.stop()
    woke, later = run(True)
    assert 4 <= woke <= 14 * 12, woke   # armed from the 3rd scrape on; bounded per scrape
    # at most one window's worth after the last scrape: (max lead 1.5 ms + window 3 ms) / 150 us
    assert later - woke <= 32
    assert run(False) == (0, 0)


def test_scrape_period_survives_one_late_scrape(native):
    """The learnt scrape period (the pre-wake's schedule): the newest request interval that
    another recent one agrees with within 12 %, so one late scrape (a pause between a
    benchmark's warm-up and its timed window, a GC stall in the scraper) costs only its own
    pre-wake; with "the two newest must agree" it cost the next two as well."""
    ms = 1_000_000
    p = native.scrape_period_ns
    assert p([100 * ms, 100 * ms]) == 100 * ms                            # two steady periods arm it
    assert p([100 * ms]) == 0 and p([]) == 0
    assert p([190 * ms, 100 * ms, 100 * ms, 100 * ms]) == 100 * ms        # a late one does not disarm it
    assert p([100 * ms, 190 * ms, 100 * ms, 100 * ms]) == 100 * ms        # nor right after it
    assert p([50 * ms, 50 * ms, 100 * ms, 100 * ms]) == 50 * ms           # a new period wins after two
    assert p([104 * ms, 96 * ms]) == 100 * ms                             # jitter within 12 % averages
    # an 8 ms late scrape agrees within 12 %, but the median keeps the period (the mean, 102 ms,
    # put the next four expected arrivals 2 ms late: profiles/r06/session3, "00000111...")
    for k in range(4):
        iv = [100 * ms] * 4
        iv[k] = 108 * ms
        assert p(iv) == 100 * ms, iv
    assert p([101 * ms, 99 * ms, 100 * ms]) == 100 * ms
    assert p([130 * ms, 100 * ms]) == 0                                   # beyond it: no period
    assert p([10 * ms, 10 * ms, 10 * ms]) == 0                            # < 20 ms: not pre-woken


def test_prewake_survives_one_late_scrape(native):
    """End to end: after one late scrape the worker is pre-woken again.  Timing-based (a
    loaded CPU delays requests past a pre-wake window), so only that pre-waking resumes is
    asserted; the rule itself is pinned by test_scrape_period_survives_one_late_scrape."""
    c = native.EngineConfig()
    c.backend = "mock"
    c.interval_s = 0
    c.http.host = "127.0.0.1"
    c.http.port = 0
    c.http.prewake = True  # (the default since round 6: slices)
    e = native.Engine(c)
    e.start()
    try:
        e.tick(1_000_000_000)
        cl = native.ScrapeClient("127.0.0.1", e.http_port, "/metrics")
        t = time.monotonic()

        def scrape_at(dt):
            nonlocal t
            t += dt
            time.sleep(max(0.0, t - time.monotonic()))
            assert cl.scrape() > 0

        for _ in range(5):
            scrape_at(0.100)
        scrape_at(0.190)  # late
        h0 = e.stats()["http_prewake_hits"]
        for _ in range(4):
            scrape_at(0.100)
        hits = e.stats()["http_prewake_hits"] - h0
    finally:
        e.stop()
    assert hits >= 1, hits


def test_prewake_right_after_a_slightly_late_scrape(native):
    """End to end: a scrape 8 ms late (within the 12 % the period learner accepts) must not
    move the next expected arrivals.  With the mean of the agreeing intervals the next four
    scrapes arrived 2 ms before the timer (profiles/r06/session3, every driver-form run:
    "00000111111111111111"); with their median they are pre-woken again."""
    c = native.EngineConfig()
    c.backend = "mock"
    c.interval_s = 0
    c.http.host = "127.0.0.1"
    c.http.port = 0
    e = native.Engine(c)
    e.start()
    try:
        e.tick(1_000_000_000)
        cl = native.ScrapeClient("127.0.0.1", e.http_port, "/metrics")
        t = time.monotonic()

        def scrape_at(dt):
            nonlocal t
            t += dt
            time.sleep(max(0.0, t - time.monotonic()))
            assert cl.scrape() > 0

        for _ in range(5):
            scrape_at(0.100)
        scrape_at(0.108)  # late, but within 12 %
        h0 = e.stats()["http_prewake_hits"]
        for _ in range(4):
            scrape_at(0.100)
        hits = e.stats()["http_prewake_hits"] - h0
    finally:
        e.stop()
    assert hits >= 2, hits  # 4 on an idle host; the mean-based period gave 0


def _thread_cpus(name: str) -> set:
    """CPUs the first thread of this process named `name` may run on."""
    import os
    for tid in os.listdir("/proc/self/task"):
        try:
            if open(f"/proc/self/task/{tid}/comm").read().strip() == name:
                return os.sched_getaffinity(int(tid))
        except OSError:
            continue
    return set()


def test_http_worker_follows_a_steady_scrapers_rx_cpu(native):
    """follow_rx_cpu: once one steady scraper is learnt, the worker is pinned to the CPU its
    requests arrive on (SO_INCOMING_CPU: the client's own CPU on loopback) and, with no steady
    connection left, returns to its own CPU mask.  Off: never pinned."""
    import os
    import socket
    own = os.sched_getaffinity(0)
    if len(own) < 2:
        pytest.skip("needs 2+ CPUs")

    def run(follow: bool):
        c = native.EngineConfig()
        c.backend = "mock"
        c.interval_s = 0
        c.http.host = "127.0.0.1"
        c.http.port = 0
        c.http.follow_rx_cpu = follow
        e = native.Engine(c)
        e.start()
        try:
            e.tick(1_000_000_000)
            cpu = min(own)
            os.sched_setaffinity(0, {cpu})  # the scraping thread sends from one known CPU
            try:
                cl = native.ScrapeClient("127.0.0.1", e.http_port, "/metrics")
                t = time.monotonic()
                for _ in range(8):
                    t += 0.030
                    time.sleep(max(0.0, t - time.monotonic()))
                    assert cl.scrape() > 0
                pinned = _thread_cpus("gpuexp-http")
                moves = e.stats()["http_rx_cpu_moves"]
                del cl  # closes the connection: no steady scraper left
                s = socket.create_connection(("127.0.0.1", e.http_port))
                s.sendall(b"GET /metrics HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n")
                while s.recv(65536):
                    pass
                s.close()
                time.sleep(0.05)
                after = _thread_cpus("gpuexp-http")
            finally:
                os.sched_setaffinity(0, own)
            return pinned, moves, after, cpu
        finally:
            e.stop()

    pinned, moves, after, cpu = run(True)
    assert pinned == {cpu} and moves >= 1, (pinned, moves)
    assert after == own, after
    pinned, moves, after, _ = run(False)
    assert pinned == own and moves == 0 and after == own


def test_gzip_copy_follows_the_scrape_schedule(native):
    """A steady keep-alive gzip scraper (every 200 ms) against a 100 Hz sampler: once its
    period is learnt, the sampler compresses only in the ticks just before each expected
    scrape instead of every tick, and every response is still served gzip'd from the
    snapshot (the worker compresses only off-schedule requests)."""
    import http.client
    c = native.EngineConfig()
    c.backend = "mock"
    c.mock_devices = 2
    c.interval_s = 0.01
    c.serve_http = True
    c.http.host = "127.0.0.1"
    c.http.port = 0
    c.http.gzip_unsteady_hold_ns = 300_000_000
    e = native.Engine(c)
    e.start()
    try:
        conn = http.client.HTTPConnection("127.0.0.1", e.http_port, timeout=5)

        def scrape():
            conn.request("GET", "/metrics", headers={"Accept-Encoding": "gzip"})
            r = conn.getresponse()
            body = r.read()
            assert r.status == 200 and r.getheader("Content-Encoding") == "gzip"
            assert gzip.decompress(body).startswith(b"# HELP")

        while e.stats()["ticks"] < 2:
            time.sleep(0.01)
        t_next = time.monotonic()
        for i in range(22):
            if i == 10:  # steady since the 5th scrape, unsteady hold (300 ms) over
                s0 = e.stats()
            scrape()
            t_next += 0.2
            time.sleep(max(0.0, t_next - time.monotonic()))
        s1 = e.stats()
        ticks = s1["ticks"] - s0["ticks"]
        eager = s1["gzip_eager"] - s0["gzip_eager"]
        on_demand = s1["http_gzip_on_demand"] - s0["http_gzip_on_demand"]
        print("ticks", ticks, "eager", eager, "on_demand", on_demand)
        # 12 scrapes over ~240 ticks: ~3 compressing ticks per scrape, not every tick
        assert ticks > 150 and eager < 0.35 * ticks, (ticks, eager)
        assert on_demand <= 3, on_demand
    finally:
        e.stop()


def _window_hits(native, arrivals, **kw):
    w = native.spin_windows(arrivals, **kw)
    inside = [bool(k) and f <= a <= u for (f, u, k), a in zip(w, arrivals[1:])]
    return w, inside


def test_spin_predictor_follows_a_relative_scraper(native):
    """A scraper that sleeps one period after each scrape (bench.py's step pacing): each
    interval is the period plus a sleep overshoot, so the next arrival is the last one plus
    the (median) period.  After 8 errors the spin window is the observed error range plus a
    margin -- far shorter than the 300 us cap on a steady client -- and holds the arrival."""
    import random
    rng = random.Random(7)
    t, arr = 10 ** 12, []
    for _ in range(120):
        t += 100_000_000 + rng.randint(40_000, 60_000)
        arr.append(t + int(rng.gauss(0, 5_000)))
    w, inside = _window_hits(native, arr)
    late = inside[20:]
    assert sum(late) / len(late) >= 0.9, sum(late) / len(late)
    assert all(k == 1 for *_, k in w[20:]) or sum(1 for *_, k in w[20:] if k == 2) < len(w[20:])
    widths = [u - f for f, u, k in w[20:]]
    assert max(widths) <= 300_000 and sorted(widths)[len(widths) // 2] < 120_000, widths[:5]


def test_spin_predictor_locks_to_a_ticker_phase(native):
    """A ticker scraper (Prometheus' scrape loop) on a busy host: scrapes land on a fixed
    grid k * period, but one in four is delayed 300 us and the next comes back on the grid.
    The relative prediction (last + period) is then off by 300 us after every late one; the
    phase-locked one is not, and wins on error spread."""
    import random
    rng = random.Random(3)
    arr = [10 ** 12 + k * 100_000_000 + (300_000 if k % 4 == 3 else 0) + int(rng.gauss(0, 5_000))
           for k in range(120)]
    w, inside = _window_hits(native, arr)
    assert sum(1 for *_, k in w[30:] if k == 2) >= 0.9 * len(w[30:])  # phase-locked chosen
    on_grid = [h for h, a in zip(inside[30:], range(31, 120)) if a % 4 != 3]
    assert sum(on_grid) / len(on_grid) >= 0.9, sum(on_grid) / len(on_grid)
    assert native.spin_windows([]) == [] and native.spin_windows([5]) == []
    # no period yet: no window
    assert native.spin_windows([10 ** 12, 10 ** 12 + 10 ** 8])[0][2] == 0


def test_prewake_mode_switches_at_run_time(native):
    """set_prewake_mode on a running engine (what SIGUSR1 + the runtime file do in the
    exporter): spin windows are entered only in spin mode, the timer stays quiet when off,
    and the spin counters reach the exposition."""
    c = native.EngineConfig()
    c.backend = "mock"
    c.interval_s = 0
    c.http.host = "127.0.0.1"
    c.http.port = 0
    assert c.http.prewake_mode == "slices"  # the default (profiles/r06/prewake_ab.md)
    c.http.prewake_mode = "off"
    e = native.Engine(c)
    e.start()
    try:
        assert e.prewake_mode == "off"
        e.tick(1_000_000_000)
        cl = native.ScrapeClient("127.0.0.1", e.http_port, "/metrics")
        t = time.monotonic()

        def scrape_n(k):
            nonlocal t
            for _ in range(k):
                t += 0.030
                time.sleep(max(0.0, t - time.monotonic()))
                assert cl.scrape() > 0

        scrape_n(12)
        s0 = e.stats()
        assert s0["http_prewake_timer_wakeups"] == 0 and s0["http_prewake_spins"] == 0
        assert e.set_prewake_mode("spin") and e.prewake_mode == "spin"
        scrape_n(20)
        s1 = e.stats()
        assert s1["http_prewake_spins"] >= 5, s1
        assert s1["http_prewake_spin_hits"] + s1["http_prewake_spin_timeouts"] <= s1["http_prewake_spins"]
        # a window is at most prewake_spin_max_ns (+ the poll's own granularity) long
        assert s1["http_prewake_spin_ns"] <= s1["http_prewake_spins"] * 400_000
        e.set_prewake_mode("off")
        scrape_n(3)
        s2 = e.stats()
        scrape_n(10)
        s3 = e.stats()
        assert s3["http_prewake_spins"] == s2["http_prewake_spins"]
        with pytest.raises(ValueError):
            e.set_prewake_mode("fast")
        e.tick(2_000_000_000)
        fams = promtext.parse(e.snapshot_text())
        assert promtext.value(fams, "gpuexp_http_prewake_spins_total", outcome="hit") == s3["http_prewake_spin_hits"]
        assert "gpuexp_http_prewake_spin_seconds_total" in fams
    finally:
        e.stop()


def _ticks_in(body: bytes) -> float:
    for line in body.decode().splitlines():
        if line.startswith("gpuexp_ticks_total"):
            return float(line.split()[-1])
    raise AssertionError("no gpuexp_ticks_total")


@pytest.mark.parametrize("when_due", [True, False])
def test_render_when_due_skips_unread_ticks_and_serves_fresh(native, when_due):
    """A steady scraper at 4 Hz against a 100 Hz sampler: with render_when_due the ticks no
    scrape will read publish nothing (most of them), yet every scrape after the period is learnt
    reads a snapshot at most 3 ticks old; without it every tick renders."""
    c = native.EngineConfig()
    c.backend = "mock"
    c.interval_s = 0.01
    c.series_profile = "standard"
    c.render_when_due = when_due
    h = c.http
    h.host = "127.0.0.1"
    h.port = 0
    c.http = h
    e = native.Engine(c)
    e.start()
    try:
        time.sleep(0.3)
        cl = native.ScrapeClient("127.0.0.1", e.http_port, "/metrics", True, 5000, "", False)
        lags = []
        t = time.perf_counter()
        s0 = None
        for i in range(16):
            assert cl.scrape(), cl.last_status
            ticks_now = e.stats()["ticks"]
            if i >= 6:
                lags.append(ticks_now - _ticks_in(gzip.decompress(cl.last_body())))
            if i == 5:
                s0 = e.stats()
            t += 0.25
            time.sleep(max(0.0, t - time.perf_counter()))
        s1 = e.stats()
    finally:
        e.stop()
    skipped = s1["renders_skipped"] - s0["renders_skipped"]
    ticks = s1["ticks"] - s0["ticks"]
    print(f"render_when_due={when_due}: {skipped} of {ticks} ticks not rendered; lag in ticks {lags}")
    assert max(lags) <= 3, lags  # (the tick counter in the body is the render's own tick)
    if when_due:
        assert skipped > 0.6 * ticks, (skipped, ticks)
    else:
        assert skipped == 0


def test_render_when_due_resumes_for_an_irregular_scraper_and_a_quiet_one(native):
    """render_when_due keeps every tick rendered (1) while an open connection without a learnt
    period has scraped, even next to a steady scraper, and (2) once the steady scraper is overdue;
    right after a steady scraper's request most ticks until its next one are skipped."""
    c = native.EngineConfig()
    c.backend = "mock"
    c.interval_s = 0.01
    c.series_profile = "compact"
    h = c.http
    h.host = "127.0.0.1"
    h.port = 0
    c.http = h
    e = native.Engine(c)
    e.start()
    try:
        time.sleep(0.2)
        steady = native.ScrapeClient("127.0.0.1", e.http_port, "/metrics", False, 5000, "", False)
        t = time.perf_counter()
        for i in range(6):  # a 3 Hz scraper: learnt after its third request
            if i:
                t += 0.33
                time.sleep(max(0.0, t - time.perf_counter()))
            assert steady.scrape()

        def skipped_over(seconds):
            s0 = e.stats()
            time.sleep(seconds)
            s1 = e.stats()
            return s1["renders_skipped"] - s0["renders_skipped"], s1["ticks"] - s0["ticks"]

        # the steady case, right after its scrape: until the next is due most ticks are skipped
        sk, n = skipped_over(0.2)
        assert 0.5 * n < sk, (sk, n)
        # (1) an irregular second connection: one request, kept open -> every tick renders
        odd = native.ScrapeClient("127.0.0.1", e.http_port, "/metrics", False, 5000, "", False)
        assert odd.scrape() and steady.scrape()
        sk, n = skipped_over(0.5)
        assert sk == 0, (sk, n)
        del odd  # closes it: the steady scraper alone again
        time.sleep(0.05)
        assert steady.scrape()
        # (2) the steady scraper stops: overdue after ~one period -> every tick renders
        time.sleep(0.8)
        sk, n = skipped_over(0.5)
        assert sk == 0, (sk, n)
    finally:
        e.stop()


def test_render_when_due_still_renders_once_a_second(native):
    """A steady scraper every 1.5 s: between its requests the engine still renders at least
    once a second (the snapshot an unexpected request reads is never older than that)."""
    c = native.EngineConfig()
    c.backend = "mock"
    c.interval_s = 0.02
    c.series_profile = "compact"
    h = c.http
    h.host = "127.0.0.1"
    h.port = 0
    c.http = h
    e = native.Engine(c)
    e.start()
    try:
        time.sleep(0.2)
        cl = native.ScrapeClient("127.0.0.1", e.http_port, "/metrics", False, 5000, "", False)
        t = time.perf_counter()
        for i in range(4):
            if i:
                t += 1.5
                time.sleep(max(0.0, t - time.perf_counter()))
            assert cl.scrape()
        s0 = e.stats()
        time.sleep(1.3)  # before the next request is due (1.5 s - two ticks)
        s1 = e.stats()
    finally:
        e.stop()
    rendered = (s1["ticks"] - s0["ticks"]) - (s1["renders_skipped"] - s0["renders_skipped"])
    assert 1 <= rendered <= 3, (rendered, s1["ticks"] - s0["ticks"])
