"""Native scrape client (bench harness): reads each response straight into one reusable
buffer — bodies must come back byte-exact across keep-alive scrapes, growing bodies,
and HTTP/1.0 servers that delimit the body by EOF (prometheus_client's)."""
import http.server
import threading


def test_keepalive_bodies_exact_and_growing(native, mock_engine):
    small = mock_engine(1)
    small.tick(1_000_000_000)
    big = mock_engine(8)
    big.tick(1_000_000_000)
    for e in (small, big):
        c = native.ScrapeClient("127.0.0.1", e.http_port, "/metrics", False, 5000)
        for _ in range(3):
            assert c.scrape() > 0
            assert c.last_status == 200 and c.errors == 0
            body = c.last_body()
            assert body.decode() == e.snapshot_text()
            assert c.last_bytes == len(body)
    def device_part(e):  # the exporter's own families do not scale with GPUs
        return sum(len(ln) + 1 for ln in e.snapshot_text().splitlines() if "gpuexp_" not in ln)
    assert device_part(big) > 3 * device_part(small)


def test_gzip_body(native, mock_engine):
    import gzip
    e = mock_engine(2)
    e.tick(1_000_000_000)
    c = native.ScrapeClient("127.0.0.1", e.http_port, "/metrics", True, 5000)
    c.scrape()            # first ask: the sampler starts pre-compressing from the next tick
    e.tick(2_000_000_000)
    assert c.scrape() > 0
    assert gzip.decompress(c.last_body()).decode() == e.snapshot_text()


class _Http10(http.server.BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.0"
    body = b"# TYPE x gauge\nx 1\n" * 5000   # ~95 KB, no Content-Length

    def do_GET(self):
        self.send_response(200)
        self.send_header("Content-Type", "text/plain")
        self.end_headers()
        self.wfile.write(self.body)

    def log_message(self, *a):
        pass


def test_http10_body_to_eof(native):
    srv = http.server.HTTPServer(("127.0.0.1", 0), _Http10)
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    try:
        c = native.ScrapeClient("127.0.0.1", srv.server_address[1], "/metrics", False, 5000)
        for _ in range(2):  # reconnects after each EOF-delimited response
            assert c.scrape() > 0
            assert c.last_body() == _Http10.body
        assert c.errors == 0
    finally:
        srv.shutdown()
