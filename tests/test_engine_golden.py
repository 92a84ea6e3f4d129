"""The engine's exposition on a deterministic mock 8-GPU node (tests/golden_engine.py), full
profile, both expositions, compared byte for byte with checked-in goldens (clock-driven values
masked).  Pins the output across refactors of the engine (round 6: engine.cc split by source,
table-driven families).  Regenerate deliberately with GPUEXP_REGEN_GOLDEN=1."""
import os

import pytest

import golden_engine

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("exposition", ["classic", "compiled"])
def test_engine_exposition_matches_golden(native, exposition):
    got = golden_engine.mask(golden_engine.run(native, exposition))
    path = os.path.join(HERE, "golden", f"engine_8gpu_full_{exposition}.txt")
    if os.environ.get("GPUEXP_REGEN_GOLDEN") == "1":
        with open(path, "w") as fh:
            fh.write(got)
    with open(path) as fh:
        want = fh.read()
    if got != want:
        import difflib
        diff = "\n".join(list(difflib.unified_diff(want.split("\n"), got.split("\n"), "golden", "now",
                                                   lineterm=""))[:60])
        pytest.fail("exposition differs from the golden:\n" + diff)


@pytest.mark.parametrize("exposition", ["classic", "compiled"])
def test_skipped_ticks_render_the_same_exposition(native, exposition):
    """render_when_due's skipped ticks write nothing to the series table but run every
    computation (rates, per-pod integration of energy / busy time / xGMI bytes, KFD event
    totals, histograms): rendering only every 3rd tick gives, on the ticks it renders, the
    exposition an every-tick engine gives (only the render counters themselves differ)."""
    import re
    every = golden_engine.mask(golden_engine.run(native, exposition, ticks=6))
    third = golden_engine.mask(golden_engine.run(native, exposition, ticks=6, render_every=3))

    def samples(t):  # (the compiled body's field widths follow its own layout history: compare values)
        t = "\n".join(" ".join(l.split()) for l in t.split("\n")
                      if not re.match(r"gpuexp_exposition_events_total\{", l))
        return t
    assert samples(every) == samples(third)
    assert 'gpuexp_exposition_events_total{event="render_skipped"}' in third or exposition == "classic"
