"""The fixed-layout exposition (SeriesTable::render_compiled, csrc/gpuexp/deflate_tmpl.cc):
every tick it must parse to exactly the samples the classic renderer gives, and its gzip
member must inflate (Python's zlib, an independent inflater) to exactly its text -- through
value churn, series appearing and going, values outgrowing their fields, histograms and
escaped labels.  Reference counterpart: promhttp's render + gzip on every scrape
(/root/reference/main.go:68-70)."""
import gzip
import math
import random
import zlib

import pytest

from kubernetes_gpu_exporter_amd.utils import promtext


def _same(a, b):
    """promtext.parse results equal, NaN == NaN."""
    assert a.keys() == b.keys()
    for name in a:
        fa, fb = a[name], b[name]
        assert fa.type == fb.type and fa.help == fb.help, name
        sa = sorted(fa.samples, key=lambda s: (s[0], sorted(s[1].items())))
        sb = sorted(fb.samples, key=lambda s: (s[0], sorted(s[1].items())))
        assert len(sa) == len(sb), name
        for (na, la, va), (nb, lb, vb) in zip(sa, sb):
            assert na == nb and la == lb, (na, la, nb, lb)
            assert va == vb or (math.isnan(va) and math.isnan(vb)), (na, la, va, vb)


def _tables(native, nfam=24):
    out = []
    for _ in range(2):
        t = native.SeriesTable()
        ids = []
        for i in range(nfam):
            ty = (native.MetricType.gauge, native.MetricType.counter)[i % 2]
            ids.append(t.add_family(f"m{i:02d}_metric_{'x' * (i % 5)}", f"help of family {i}: \\ and \n", ty, ["gpu", "k"]))
        h = t.add_family("lat_seconds", "a histogram", native.MetricType.histogram, ["gpu"])
        out.append((t, ids, h))
    return out


def _value(rng, gen):
    return rng.choice([rng.random() * 1000, float(rng.randint(0, 10 ** rng.randint(1, 15))), 0.0, -3.25,
                       float("nan"), float("inf"), float("-inf"), gen * 1.5, 1e-300, 2.0 ** 60])


@pytest.mark.parametrize("churn", [0.0, 0.05])
def test_compiled_matches_classic_every_tick(native, churn):
    (a, ia, ha), (b, ib, hb) = _tables(native)
    rng = random.Random(7)
    for gen in range(1, 120):
        for i in range(len(ia)):
            for g in range(8):
                for k in ("a", 'q"\\z\n') if i % 3 == 0 else ("a",):
                    if gen > 1 and rng.random() < churn:
                        continue  # not set this tick: gone (gc_after 1) -> the family is laid out again
                    v = _value(rng, gen) if rng.random() < 0.5 else float(g)
                    a.put(ia[i], [str(g), k], v, gen)
                    b.put(ib[i], [str(g), k], v, gen)
        for g in range(3):
            v = rng.random() * 10
            a.observe(ha, [str(g)], v, gen, [0.1, 1.0, 5.0])
            b.observe(hb, [str(g)], v, gen, [0.1, 1.0, 5.0])
        ref = a.render(gen, 1)
        txt, gz = b.render_compiled(gen, 1, True)
        _same(promtext.parse(ref), promtext.parse(txt))
        assert gzip.decompress(gz) == txt.encode(), gen
        assert zlib.decompress(gz, 31) == txt.encode()  # zlib's own inflater, gzip wrapper
    if churn == 0.0:  # values settle in their widths: a real parse and a code of its own happen
        assert b.code_builds() >= 2, b.code_builds()


def test_steady_state_does_not_relayout(native):
    (t, ids, h), _ = _tables(native, 8)
    for gen in range(1, 60):
        for i, f in enumerate(ids):
            for g in range(4):
                # same text length every tick (3-digit integers): fields never grow
                t.put(f, [str(g), "a"], float(100 + (gen * 7 + i + g) % 900), gen)
        txt, gz = t.render_compiled(gen, 1, True)
        if gen > 1:
            assert t.last_relayouts() == 0, gen
        assert gzip.decompress(gz) == txt.encode()
    assert t.code_builds() == 2  # one for the first (literal) encodes, one after the real parse


def test_unchanged_families_are_passed_over(native):
    """A family whose laid-out members were all set again with the same values is passed over
    without walking its members; one changed value is still patched, a skipped generation
    (a publish without a render) forces a full pass, and a member gone stale is noticed."""
    (t, ids, h), _ = _tables(native, 6)
    for gen in range(1, 5):
        for f in ids:
            for g in range(3):
                t.put(f, [str(g), "a"], float(g), gen)
        t.render_compiled(gen, 1, True)
    assert t.last_skipped() == len(ids)
    for f in ids:
        for g in range(3):
            t.put(f, [str(g), "a"], 7.0 if (f == ids[2] and g == 1) else float(g), 5)
    txt, gz = t.render_compiled(5, 1, True)
    assert t.last_skipped() == len(ids) - 1
    assert promtext.value(promtext.parse(txt), "m02_metric_xx", gpu="1", k="a") == 7.0
    assert gzip.decompress(gz) == txt.encode()
    # generation 6 set but never rendered: 7 must look at every family again
    for gen, v in ((6, 8.0), (7, 8.0)):
        for f in ids:
            for g in range(3):
                t.put(f, [str(g), "a"], v if (f == ids[4] and g == 0) else float(g), gen)
    txt, gz = t.render_compiled(7, 1, True)
    assert t.last_skipped() == 0
    assert promtext.value(promtext.parse(txt), "m04_metric_xxxx", gpu="0", k="a") == 8.0
    # a member not set: its family is walked and laid out again without it
    for f in ids:
        for g in range(3):
            if not (f == ids[0] and g == 2):
                t.put(f, [str(g), "a"], float(g), 8)
    txt, gz = t.render_compiled(8, 1, True)
    assert t.last_relayouts() == 1
    assert [lab["gpu"] for _, lab, _ in promtext.parse(txt)["m00_metric_"].samples] == ["0", "1"]
    assert gzip.decompress(gz) == txt.encode()


def test_provisional_parses_while_the_layout_settles(native):
    """A family laid out again is parsed on its own (matches within its own bytes only) while the
    layout still moves; the real parse, reaching back into the families before it, comes once the
    layout held for 3 renders, and the gzip member is valid and equal to the text throughout."""
    (t, ids, h), _ = _tables(native, 4)
    gen = 0
    lit, sizes = [], []
    for v in [5.0] * 10 + [123456.0] + [5.0] * 10:
        gen += 1
        for f in ids:
            t.put(f, ["0", "a"], v if f == ids[1] else 1.0, gen)
        before = t.provisional_parses()
        txt, gz = t.render_compiled(gen, 1, True)
        lit.append(t.provisional_parses() - before)
        sizes.append(len(gz))
        assert gzip.decompress(gz) == txt.encode()
    # first layout: every family provisional; the outgrown field at 11: its family provisional again
    assert lit[0] == len(ids) and sum(lit[1:10]) == 0 and lit[10] >= 1 and sum(lit[11:]) == 0, lit
    assert sizes[9] < sizes[0]        # the real parse after the first 3 renders compresses better
    assert sizes[-1] <= sizes[10]     # ... and again after the outgrown field settled


def test_outgrown_field_relayouts_only_its_family(native):
    (t, ids, h), _ = _tables(native, 6)
    for gen in range(1, 4):
        for f in ids:
            t.put(f, ["0", "a"], 5.0, gen)
        t.render_compiled(gen, 1, True)
    for f in ids:
        t.put(f, ["0", "a"], 5.0, 4)
    t.put(ids[3], ["0", "a"], 123456789.125, 4)  # outgrows its 1-byte field
    txt, gz = t.render_compiled(4, 1, True)
    assert t.last_relayouts() == 1
    assert gzip.decompress(gz) == txt.encode()
    # back to a short value: the field keeps its width (right-aligned behind blanks; an
    # outgrown fraction field gets the room of the longest round-trip form, 24), no new layout
    for f in ids:
        t.put(f, ["0", "a"], 5.0, 5)
    txt, gz = t.render_compiled(5, 1, True)
    assert t.last_relayouts() == 0
    line = [ln for ln in txt.splitlines() if ln.startswith("m03_")][0]
    assert line.endswith("} " + " " * 23 + "5")
    # an outgrown integer field keeps two more digits of room
    for f in ids:
        t.put(f, ["0", "a"], 5.0, 6)
    t.put(ids[1], ["0", "a"], 1234.0, 6)
    t.render_compiled(6, 1, True)
    assert t.last_relayouts() == 1
    for f in ids:
        t.put(f, ["0", "a"], 5.0, 7)
    t.put(ids[1], ["0", "a"], 123456.0, 7)
    txt, gz = t.render_compiled(7, 1, True)
    assert t.last_relayouts() == 0 and gzip.decompress(gz) == txt.encode()
    assert promtext.parse(txt)["m03_metric_xxx"].samples[0][2] == 5.0
    assert gzip.decompress(gz) == txt.encode()


def test_compiled_gzip_is_close_to_zlib(native):
    """Static bytes are LZ77-parsed once per layout (matches reach back into the preceding
    families), values are literals: the member stays within ~25 % of zlib level 1 on a body
    shaped like the exporter's (many families with the same label sets)."""
    t = native.SeriesTable()
    ids = [t.add_family(f"amd_gpu_{n}", f"The {n.replace('_', ' ')} of the GPU, from the PMFW metrics table",
                        native.MetricType.gauge, ["gpu", "xcc"])
           for n in ("xcc_busy_percent", "xcc_clock_hz", "xcc_mfma_busy_percent", "xcc_temperature_celsius",
                     "xcc_power_watts", "xcc_util_percent", "xcc_waves", "xcc_lds_bytes")]
    for gen in range(1, 13):  # (the real parse comes after 3 renders of a settled layout)
        for f in ids:
            for g in range(8):
                for x in range(8):
                    t.put(f, [str(g), str(x)], float((g * 8 + x) * 37 % 101), gen)
        txt, gz = t.render_compiled(gen, 1, True)
    z1 = len(zlib.compress(txt.encode(), 1))
    assert len(gz) <= 1.25 * z1, (len(gz), z1)


def test_engine_compiled_and_classic_expose_the_same_samples(mock_engine):
    """The two engine exposition modes on the 8-GPU mock node, tick for tick."""
    a = mock_engine(8, http=False, series_profile="full", exposition="classic")
    b = mock_engine(8, http=False, series_profile="full", exposition="compiled")
    for i in range(1, 6):
        a.tick(i * 100_000_000)
        b.tick(i * 100_000_000)
        pa, pb = promtext.parse(a.snapshot_text()), promtext.parse(b.snapshot_text())
        # self-metrics (tick CPU, stage times) legitimately differ between two engines
        for p in (pa, pb):
            for name in [n for n in p if n.startswith("gpuexp_")]:
                del p[name]
        _same(pa, pb)


def test_engine_gzip_scrape_inflates_to_the_identity_body(mock_engine):
    """A gzip scrape is served from the member the sampler emitted with the body (compiled
    mode) and inflates to the identity body of the same snapshot."""
    import http.client
    e = mock_engine(2, series_profile="full")

    def get(enc):
        c = http.client.HTTPConnection("127.0.0.1", e.http_port, timeout=5)
        c.request("GET", "/metrics", headers={"Accept-Encoding": enc})
        r = c.getresponse()
        body = r.read()
        c.close()
        return r.getheader("Content-Encoding"), body

    e.tick(100_000_000)
    get("gzip")  # a gzip client: the sampler emits a gzip member with every snapshot from now on
    for i in range(2, 6):
        e.tick(i * 100_000_000)
        enc, gz = get("gzip")
        assert enc == "gzip"
        _, ident = get("identity")
        assert gzip.decompress(gz) == ident == e.snapshot_text().encode()
    assert e.stats()["gzip_eager"] >= 4


def test_compiled_randomized_layouts(native):
    """Property check (hypothesis): any family set, label values (escapes, unicode), value
    sequence and liveness pattern renders through the compiled path to exactly the classic
    renderer's samples, and its gzip member inflates to its text."""
    hypothesis = pytest.importorskip("hypothesis")
    st = hypothesis.strategies
    label = st.text(alphabet=st.characters(blacklist_categories=("Cs",)), max_size=12)
    value = st.one_of(st.floats(allow_nan=True, allow_infinity=True), st.integers(-10**15, 10**15).map(float))

    @hypothesis.settings(max_examples=40, deadline=None)
    @hypothesis.given(nfam=st.integers(1, 5), labels=st.lists(label, min_size=1, max_size=6, unique=True),
                      ticks=st.lists(st.lists(st.one_of(st.none(), value), min_size=30, max_size=30),
                                     min_size=2, max_size=16))
    def check(nfam, labels, ticks):
        a, b = native.SeriesTable(), native.SeriesTable()
        fa = [a.add_family(f"f{i}_x", f"help {i}", native.MetricType.gauge, ["l"]) for i in range(nfam)]
        fb = [b.add_family(f"f{i}_x", f"help {i}", native.MetricType.gauge, ["l"]) for i in range(nfam)]
        for gen, vals in enumerate(ticks, start=1):
            k = 0
            for i in range(nfam):
                for lab in labels:
                    v = vals[k % len(vals)]
                    k += 1
                    if v is None:
                        continue  # not set this tick
                    a.put(fa[i], [lab], v, gen)
                    b.put(fb[i], [lab], v, gen)
            ref = a.render(gen, 1)
            txt, gz = b.render_compiled(gen, 1, True)
            _same(promtext.parse(ref), promtext.parse(txt))
            assert zlib.decompress(gz, 31) == txt.encode()

    check()


def test_settling_is_per_family(native):
    """One family laid out again every few ticks (a value outgrowing, a process coming) must not
    keep the rest of the body in provisional parses: each family gets its real parse once it
    has held for 3 renders, whatever the others do (on silicon, an owner-label change re-laid 70
    families at once while a few kept moving, profiles/r05/session6)."""
    (t, ids, h), _ = _tables(native, 12)
    sizes = []
    for gen in range(1, 60):
        owner = "pod-a" if gen < 14 else "pod-b"  # every series renamed at 14 (a new owner label)
        for i, f in enumerate(ids):
            v = float(10 ** (gen // 5)) if i == 5 else 1.0  # family 5 outgrows its field every 5 ticks
            for g in range(4):
                t.put(f, [str(g), owner], v, gen)
        txt, gz = t.render_compiled(gen, 1, True)
        assert gzip.decompress(gz) == txt.encode()
        sizes.append(len(gz))
    settled_before, all_provisional = sizes[12], sizes[14]
    # a provisional parse still compresses (matches within the family: its label sets repeat)
    assert all_provisional < 0.5 * len(txt), (all_provisional, len(txt))
    # family 5 (field room: one extra digit) is laid out again at 25 and 40; only it is
    # provisional meanwhile, and everything else -- including the segments whose matches had to
    # stop short of it -- gets its full parse back once it settles (gens 33..39)
    assert max(sizes[24:32]) < 0.6 * all_provisional, (all_provisional, sizes[24:32])
    assert max(sizes[32:39]) < 1.05 * settled_before, (settled_before, sizes[32:39])


def test_compiled_randomized_settling(native):
    """Property check (hypothesis) of the settling policy: families disturbed on a random schedule
    (a value outgrowing its field, a series gone for a tick, every series renamed), gzip asked for
    on random ticks only.  Every gzip member inflates to its text, every text parses to the
    classic renderer's samples, and once the body has been quiet for 10 renders its gzip is as
    small as a fresh table's settled one: no segment is left provisional or cut short."""
    hypothesis = pytest.importorskip("hypothesis")
    st = hypothesis.strategies
    event = st.tuples(st.integers(1, 30), st.integers(0, 7), st.sampled_from(["outgrow", "drop", "rename"]))

    def state(nfam, evs, gen):
        """{(family, label): value} at `gen` under the events so far."""
        out = {}
        for i in range(nfam):
            mine = [(t, k) for t, f, k in evs if f % nfam == i and t <= gen]
            grow = sum(1 for t, k in mine if k == "outgrow")
            owner = "own-%d" % sum(1 for t, k in mine if k == "rename")
            gone = any(t == gen and k == "drop" for t, k in mine)
            for g in range(3):
                if not (gone and g == 1):
                    out[(i, (str(g), owner))] = float(10 ** (2 * grow)) + g
        return out

    @hypothesis.settings(max_examples=30, deadline=None)
    @hypothesis.given(nfam=st.integers(2, 8), evs=st.lists(event, max_size=12),
                      want=st.lists(st.booleans(), min_size=45, max_size=45))
    def check(nfam, evs, want):
        a, b, c = native.SeriesTable(), native.SeriesTable(), native.SeriesTable()
        fams = [[t.add_family(f"f{i}_metric_seconds", f"help of {i}", native.MetricType.gauge, ["gpu", "pod"])
                 for i in range(nfam)] for t in (a, b, c)]
        last = None
        for gen in range(1, 46):
            for (i, labs), v in state(nfam, evs, gen).items():
                a.put(fams[0][i], list(labs), v, gen)
                b.put(fams[1][i], list(labs), v, gen)
            ref = a.render(gen, 1)
            txt, gz = b.render_compiled(gen, 1, want[gen - 1] or gen > 40)
            _same(promtext.parse(ref), promtext.parse(txt))
            if gz:
                assert zlib.decompress(gz, 31) == txt.encode(), gen
                last = gz
        # a fresh table given the final state from the start, settled the same way
        for gen in range(1, 12):
            for (i, labs), v in state(nfam, evs, 45).items():
                c.put(fams[2][i], list(labs), v, gen)
            _, fresh = c.render_compiled(gen, 1, True)
        assert len(last) <= 1.1 * len(fresh) + 16, (len(last), len(fresh))

    check()


@pytest.mark.parametrize("gc_after", [1, 3])
def test_rotating_slots_take_only_the_changed_fields(native, gc_after):
    """The engine renders into rotating snapshot slots (render_compiled with out_gen): a slot
    that holds this layout's body as of an older generation gets only the fields changed
    since then copied in.  With 3 slots, skipped generations (a publish that did not happen),
    relayouts (a value outgrowing its field, series coming and going), families passed over
    unchanged and gc_after > 1, every slot's text must equal a fresh render of a twin table
    with the same history, and its gzip must inflate to it (a stale field left in
    a rotating slot would publish wrong values under a valid gzip)."""
    rng = random.Random(11 + gc_after)
    a, b = native.SeriesTable(), native.SeriesTable()
    nfam = 7
    fa = [a.add_family(f"s{i}_metric", f"help {i}", native.MetricType.gauge, ["gpu", "k"]) for i in range(nfam)]
    fb = [b.add_family(f"s{i}_metric", f"help {i}", native.MetricType.gauge, ["gpu", "k"]) for i in range(nfam)]
    vals = {}
    gen = 0
    copied_less = 0
    for step in range(160):
        gen += 2 if rng.random() < 0.15 else 1  # a skipped generation now and then
        for i in range(nfam):
            if i == 0 and step:
                # family 0: the same series every tick, values changed every 3rd (else passed over)
                for (fi, g, k), v in [(k, v) for k, v in vals.items() if k[0] == 0]:
                    v = float(rng.randint(0, 99)) if step % 3 == 0 else v
                    vals[(fi, g, k)] = v
                    a.put(fa[fi], [g, k], v, gen)
                    b.put(fb[fi], [g, k], v, gen)
                continue
            churn = step % 12 == 0  # layout changes come in bursts, steady ticks in between
            for g in range(3):
                if churn and rng.random() < 0.2:
                    continue  # series absent this tick (GC'd after gc_after generations)
                key = (i, str(g), "y" if churn and rng.random() < 0.2 else "x")  # sometimes a new series
                r = rng.random()
                if r < 0.6 and key in vals:
                    v = vals[key]  # unchanged
                elif r < 0.97 or not churn:
                    v = float(rng.randint(0, 99))
                else:
                    v = float(rng.randint(0, 10 ** rng.randint(3, 12)))  # may outgrow its field
                vals[key] = v
                a.put(fa[i], [key[1], key[2]], v, gen)
                b.put(fb[i], [key[1], key[2]], v, gen)
        txt, gz, copied = a.render_compiled_slot(gen, gen % 3, gc_after)
        ref, _ = b.render_compiled(gen, gc_after, False)
        assert txt == ref, (step, gen)
        assert zlib.decompress(gz, 31) == txt.encode()
        if copied < len(txt):
            copied_less += 1
    assert copied_less > 40  # the delta path really ran (not only full copies)
