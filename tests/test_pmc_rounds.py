"""The aqlprofile plugin's read machine (csrc/gpuexp/pmc_rounds.{h,cc}) on 8 scripted fake GPUs
(csrc/gpuexp/pmc_fake.h): the round / rescue / probation / re-arm / leftover state machine that
aql_pmc.cc drives on HSA queues, exercised on the CPU before an 8-GPU node ever runs it.

A fake GPU's reads complete after a scripted latency; its first queue can stand still for a
while (a sentinel dispatch the workload leaves no wave slot for), its counters can be reset or
stopped by "another profiler", and its queue can fail.  The harness drives the machine the way
the engine drives the plugin (kick, device reads, sync, sample every GPU) while a reader thread
calls the readers concurrently, and reports per GPU: the health counters, the windows published,
whether each window's rates were right, and per read packet when it completed / was first looked
at / was seen, and how often its output was collected.  The same scenarios run under TSan and
ASan+UBSan in tests/test_sanitizers.py (csrc/tests/pmc_harness_main.cc).

Reference counterpart: the per-device loop /root/reference/main.go:123-138 (one device's failure
there is fatal for all of them, log.Fatalf at main.go:126/131/137).
"""
import threading

import pytest

MS = 1000  # script times are microseconds
JITTER_US = 30000  # OS scheduling jitter allowed on top of one polling slice (sleep overshoot; xdist load)


def run(native, **kw):
    cfg = {"gpus": 8, "ticks": 80, "tick_us": 20000, "work_us": 300, "sync_us": 2000, "rearm_base_ms": 100,
           "rate_tolerance": 0.4}
    cfg.update(kw)
    return native.pmc_harness(cfg)


def _hiccup_bound(r, stalled):
    """Worst rate error allowed for the stalled GPU: 10 %, or the healthy GPUs' worst plus 5
    points when the harness thread itself was descheduled (that hits every GPU at once)."""
    others = [g["worst_rate_err"] for i, g in enumerate(r["gpus"]) if i != stalled and not g["broken"]]
    return max(0.1, max(others) + 0.05)


def healthy(g, ticks):
    assert g["double_collected"] == 0 and g["uncollected"] == 0
    assert g["bad_windows"] == 0, g
    assert g["stalls"] == 0 and g["rescues"] == 0 and g["resets"] == 0 and not g["broken"]
    # (a window whose ends are timed worse than 5 % of it -- a look delayed by scheduling on this
    # shared CPU -- is merged into the next one rather than published: a few may be missing)
    assert g["windows"] >= ticks - 5 and g["fresh_ticks"] >= 0.85 * ticks, g


# ---------------------------------------------------------------------------------------------
# the back-off decision (counter_model.h rearm_on_reset / rearm_due / rearm_done)
# ---------------------------------------------------------------------------------------------
def test_rearm_backoff_doubles_while_someone_keeps_resetting(native):
    # (a reset within 2 back-offs of our own arm would count as a conflict at once: see below)
    st = native.rearm_policy([(0, "armed"), (5000, "backwards"), (5500, "check"), (6100, "check"),
                              (6200, "backwards"), (6300, "backwards"), (9000, "check"), (10400, "check"),
                              (10400, "armed")], base_ms=1000, max_ms=8000)
    waiting, due, backoff, conflicts, due_now = zip(*st)
    assert st[1][:4] == (True, 6000.0, 1000.0, 0)      # first reset: wait one base back-off
    assert due_now[2] is False and due_now[3] is True    # not before, due after
    assert st[4][1:4] == (8200.0, 2000.0, 1)            # reset while waiting: doubled, from now
    assert st[5][1:4] == (10300.0, 4000.0, 2)
    assert due_now[6] is False and due_now[7] is True
    assert waiting[8] is False                           # re-armed


def test_rearm_backoff_stopped_counters_do_not_extend_and_conflict_after_rearm_doubles(native):
    st = native.rearm_policy([(0, "armed"), (10000, "stopped"), (10500, "stopped"), (11001, "check"),
                              (11001, "armed"), (11500, "backwards")], base_ms=1000, max_ms=64000)
    assert st[1][:3] == (True, 11000.0, 1000.0)
    assert st[2][:3] == (True, 11000.0, 1000.0)          # stopped again: nobody counts, no extension
    assert st[3][4] is True
    # reset 0.5 s after our re-arm: the other profiler is still there -> double
    assert st[5][:4] == (True, 13500.0, 2000.0, 1)


def test_rearm_backoff_is_capped_and_calms_down(native):
    ev = [(0, "armed")] + [(1000 + 10 * i, "backwards") for i in range(12)]
    st = native.rearm_policy(ev, base_ms=1000, max_ms=8000)
    assert st[-1][2] == 8000.0                           # capped
    st = native.rearm_policy([(0, "armed"), (1000, "backwards"), (1100, "backwards"), (4000, "armed"),
                              (400000, "backwards")], base_ms=1000, max_ms=8000, calm_ms=300000)
    assert st[-1][2] == 1000.0                           # long after the last re-arm: base again


def test_rearm_modes_off_and_now(native):
    off = native.rearm_policy([(0, "armed"), (10, "backwards"), (1e7, "check")], mode="off")
    assert off[-1][0] is True and off[-1][4] is False    # waits for ever
    now = native.rearm_policy([(0, "armed"), (10, "backwards"), (10, "check")], mode="now")
    assert now[-1][4] is True                            # round-4 behaviour: at once


# ---------------------------------------------------------------------------------------------
# the machine on fake GPUs
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("inline", [True, False], ids=["inline", "thread"])
def test_stuck_gpu_never_holds_the_other_seven(native, inline):
    # reads complete between 50 us and 610 us after posting, so most complete while a sync looks
    scripts = [{"latency_us": 50 + 80 * i} for i in range(8)]
    scripts[3]["stalls"] = [(200 * MS, 800 * MS)]
    r = run(native, inline=inline, scripts=scripts)
    assert r["armed_all"]
    for i, g in enumerate(r["gpus"]):
        if i == 3:
            continue
        healthy(g, r["ticks"])
        # seen within one polling slice of completing (or at the first look), whatever GPU 3 does
        assert g["max_lateness_us"] <= 100 + JITTER_US, (i, g)
    if inline:
        # only the round in which GPU 3 first stuck waits out the sync; afterwards its read gets one
        # look per round and the sync returns as soon as the others are in
        assert r["late_syncs"] <= 2, r
    g3 = r["gpus"][3]
    assert g3["stalls"] >= 3 and g3["rescues"] == 1 and g3["releases"] == 1
    assert g3["rescue_opened"] == g3["rescue_closed"] == 1 and not g3["rescue_open_at_end"] and g3["misuse"] == 0
    assert not g3["rescue_active"]
    assert g3["double_collected"] == 0 and g3["uncollected"] == 1   # the read abandoned on queue 0
    assert g3["bad_windows"] == 0 and g3["worst_rate_err"] < _hiccup_bound(r, 3), g3
    # the rescue queue kept GPU 3's windows coming during most of the 600 ms stall
    assert g3["windows"] >= r["ticks"] - 8, g3


def test_leftover_reads_are_collected_exactly_once(native):
    # GPU 1's reads take 3 ms, the sync waits 1 ms: every round leaves its read to the counting
    # thread, which collects it (or the next kick's one look does)
    scripts = [{} for _ in range(8)]
    scripts[1]["latency_us"] = 3000
    r = run(native, inline=True, sync_us=1000, scripts=scripts)
    assert r["late_syncs"] >= r["ticks"] // 2  # (a sync that starts late, OS jitter, finds it done)
    g1 = r["gpus"][1]
    assert g1["double_collected"] == 0 and g1["uncollected"] == 0
    assert g1["reads_completed"] >= r["ticks"] - 2  # (counted up to two ticks before the stop)
    # (a read collected after the sync is timed only to within the counting thread's look: the
    # few whose look came late are merged into the next window rather than published mistimed)
    assert g1["windows"] >= r["ticks"] - 12 and g1["bad_windows"] == 0
    assert g1["stalls"] == 0  # seen complete before the next round's one look
    for i in (0, 2, 3, 4, 5, 6, 7):
        healthy(r["gpus"][i], r["ticks"])


def test_foreign_reset_rearms_exactly_once(native):
    scripts = [{} for _ in range(8)]
    scripts[2]["resets"] = [300 * MS]
    r = run(native, scripts=scripts)
    g2 = r["gpus"][2]
    assert g2["resets"] == 1 and g2["rearms"] == 1 and g2["arms"] == 1 and g2["conflicts"] == 0
    assert not g2["waiting_rearm"] and g2["bad_windows"] == 0
    # withheld from the reset until the re-arm (~100 ms back-off), then back
    assert r["ticks"] - 12 <= g2["windows"] <= r["ticks"] - 3, g2
    for i in (0, 1, 3, 4, 5, 6, 7):
        healthy(r["gpus"][i], r["ticks"])


def test_another_profiler_is_not_fought(native):
    # someone resets the counters every 50 ms for 150 ms: every reset doubles the back-off and
    # moves the re-arm out; the exporter re-arms once, 800 ms after the last one
    scripts = [{} for _ in range(8)]
    scripts[4]["resets"] = [300 * MS, 350 * MS, 400 * MS, 450 * MS]
    r = run(native, ticks=90, scripts=scripts)
    g4 = r["gpus"][4]
    assert g4["resets"] == 4 and g4["conflicts"] == 3 and g4["rearms"] == 1 and g4["arms"] == 1, g4
    assert g4["bad_windows"] == 0
    assert g4["windows"] <= r["ticks"] - 40  # withheld ~0.3 .. ~1.26 s


@pytest.mark.parametrize("mode,rearms,waiting", [("off", 0, True), ("now", 1, False)])
def test_rearm_modes_on_the_machine(native, mode, rearms, waiting):
    scripts = [{} for _ in range(8)]
    scripts[2]["resets"] = [300 * MS]
    # "now" re-arms inside the round that saw the reset: the next window's start is the arm's
    # completion, estimated to half a polling interval -- on a loaded CPU (xdist) a 20 ms window
    # can be off by more than the default 40 %
    r = run(native, rearm=mode, scripts=scripts, rate_tolerance=0.6)
    g2 = r["gpus"][2]
    assert g2["rearms"] == rearms and g2["waiting_rearm"] is waiting and g2["bad_windows"] == 0
    if mode == "now":
        assert g2["windows"] >= r["ticks"] - 4  # re-armed at the next round
    else:
        assert g2["windows"] <= 300 * MS // 20000 + 1  # nothing after the reset


def test_counters_stopped_by_someone_else_are_rearmed(native):
    scripts = [{} for _ in range(8)]
    scripts[5]["stops"] = [(300 * MS, -1)]
    r = run(native, scripts=scripts)
    g5 = r["gpus"][5]
    assert g5["resets"] == 1 and g5["rearms"] == 1 and not g5["waiting_rearm"], g5


def test_queue_error_is_isolated(native):
    scripts = [{} for _ in range(8)]
    scripts[6]["queue_error_at"] = 500 * MS
    r = run(native, scripts=scripts)
    g6 = r["gpus"][6]
    assert g6["broken"] and g6["windows"] <= 500 * MS // 20000 + 1
    for i in (0, 1, 2, 3, 4, 5, 7):
        healthy(r["gpus"][i], r["ticks"])


def test_rescue_unavailable_only_stalls(native):
    scripts = [{} for _ in range(8)]
    scripts[3].update(stalls=[(200 * MS, 600 * MS)], rescue_fails=True)
    r = run(native, scripts=scripts)
    g3 = r["gpus"][3]
    assert g3["rescues"] == 0 and g3["rescue_opened"] == 0 and g3["misuse"] == 0 and g3["stalls"] >= 10
    assert g3["double_collected"] == 0 and g3["uncollected"] == 0 and g3["bad_windows"] == 0
    assert not g3["broken"] and g3["windows"] >= r["ticks"] - 25  # back after the stall
    # the read that sat out the stall is seen complete only at the next round's look: its time is
    # uncertain by half a tick, so no window may end or start there (round 4 published a 29 % rate
    # error here; on silicon 23 % in the fp8 FLOP/s calibration, profiles/r05/session4).  The
    # stalled GPU's worst window is no worse than what a scheduling hiccup does to every GPU.
    assert g3["worst_rate_err"] < _hiccup_bound(r, 3), g3


@pytest.mark.parametrize("read_mode,mode", [(1, "resets"), (2, "stops")])
def test_non_cumulative_read_modes(native, read_mode, mode):
    r = run(native, mode=mode, ticks=40, scripts=[{"read_mode": read_mode} for _ in range(8)])
    for g in r["gpus"]:
        assert g["windows"] >= 37 and g["bad_windows"] == 0 and g["double_collected"] == 0, g


def test_eight_agents_inline_and_thread_machines_at_once(native):
    """Every behaviour on one node at once, an inline machine and a thread-mode one concurrently
    (the CPU twin of the sanitizer driver csrc/tests/pmc_harness_main.cc)."""
    scripts = [{} for _ in range(8)]
    scripts[1]["latency_us"] = 3000
    scripts[2]["resets"] = [300 * MS]
    scripts[3]["stalls"] = [(200 * MS, 800 * MS)]
    scripts[4]["resets"] = [300 * MS, 350 * MS, 400 * MS, 450 * MS]
    scripts[5]["stops"] = [(300 * MS, -1)]
    scripts[6]["queue_error_at"] = 500 * MS
    scripts[7]["latency_us"] = 400
    out = {}

    def go(inline):
        out[inline] = run(native, inline=inline, ticks=90, sync_us=1000, scripts=scripts, rate_tolerance=0.5)

    ts = [threading.Thread(target=go, args=(m,)) for m in (True, False)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for inline, r in out.items():
        g = r["gpus"]
        for i, x in enumerate(g):
            assert x["double_collected"] == 0 and x["misuse"] == 0, (inline, i, x)
            assert x["rescue_opened"] == x["rescue_closed"] and not x["rescue_open_at_end"], (inline, i, x)
            assert x["uncollected"] <= (1 if i in (3, 6) else 0), (inline, i, x)
            if i != 6:
                assert x["bad_windows"] == 0, (inline, i, x)
        for i in (0, 1, 7):  # (GPU 1's 3 ms reads outlast the sync: merged windows, more under CPU load)
            assert g[i]["windows"] >= r["ticks"] - (20 if i == 1 else 5), (inline, i, g[i])
        assert (g[2]["resets"], g[2]["rearms"], g[2]["arms"]) == (1, 1, 1)
        assert (g[3]["rescues"], g[3]["releases"]) == (1, 1) and g[3]["stalls"] >= 3
        assert (g[4]["rearms"], g[4]["conflicts"]) == (1, 3)
        assert (g[5]["resets"], g[5]["rearms"]) == (1, 1)
        assert g[6]["broken"]
        assert r["reader_calls"] > 1000


def test_hsa_port_multi_agent_lifecycle_on_stub_gpus(native):
    """The aqlprofile plugin's multi-agent bookkeeping (pmc_agents.h: BDF matching with a
    reserved agent, per-GPU setup, arm, the rescue queue's ownership, teardown) on 8 stub GPUs
    plus one the engine reserves without a queue, through the same templates aql_pmc.cc uses
    on HSA (the port had only ever run with one agent).  GPU 3's queue creation
    fails: the other 7 are armed and read; GPU 5's first queue stalls behind a sentinel run and
    its reads move to a rescue queue and back; GPU 6 is broken at teardown, so its buffers are
    left to the runtime's shutdown.  No queue or signal outlives teardown, nothing is released
    twice, and only the broken GPU's buffers are left (the sanitizer presets run the same
    lifecycle: csrc/tests/pmc_harness_main.cc)."""
    o = native.pmc_agent_lifecycle(8, 3, 5, 6, 40)
    assert o["devices"] == 9 and o["matched"] == 8, o
    assert o["usable"] == 7 and o["armed"] == 7, o
    assert o["queues_created"] == 8 and o["signals_created"] == 8, o  # 7 setups + the rescue; GPU 3 got none
    assert o["queues_live"] == 0 and o["signals_live"] == 0, o
    assert o["double_release"] == 0 and o["foreign_release"] == 0, o
    assert o["buffers_left_by_design"] == 2 and o["buffers_live"] == 2, o  # GPU 6's command + output buffers
    assert o["rescues_opened"] >= 1 and o["rescues_closed"] == o["rescues_opened"], o
    assert o["windows_on_failed_gpu"] == 0, o
    w = o["windows"]
    assert w[0] == 0  # the reserved device (listed first: the engine's order is reversed)
    assert sum(1 for x in w if x >= 30) == 7, w  # every usable GPU read on (nearly) every tick
