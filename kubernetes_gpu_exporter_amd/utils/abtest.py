"""Interleaved in-process A/B of exporter settings (bench.py --prewake-ab).

Round 5 changed the HTTP pre-wake default on five on/off pairs, each arm a separate
exporter process: a two-sided signed-rank test on n = 5 cannot go below p = 0.0625, and
box drift between processes swamped the effect (What's weak #1).  Here every
arm runs inside ONE exporter process on one box: the arms alternate every `block` timed
scrapes in a random order per round, so drift hits all arms alike, and each arm gets
hundreds of scrapes.  Differences are judged by a block bootstrap (blocks resampled with
replacement, so the within-block correlation of consecutive scrapes is kept) of the p50
and of the CPU %.

Reference: the reference renders and serves on each scrape (promhttp,
/root/reference/main.go:68-71) and has no tuning of this kind at all.
"""
from __future__ import annotations

import random
import statistics
from dataclasses import dataclass, field


def block_schedule(arms: list, n_blocks: int, seed: int = 0) -> list:
    """Arm of each of `n_blocks` blocks: rounds of every arm once, each round a fresh random
    order (a fixed rotation would line an arm up with any periodic disturbance)."""
    rng = random.Random(seed)
    out: list = []
    while len(out) < n_blocks:
        r = list(arms)
        rng.shuffle(r)
        out.extend(r)
    return out[:n_blocks]


@dataclass
class Block:
    arm: str
    scrapes: list = field(default_factory=list)  # per scrape: dict(total, req, sq, pw)
    wall_s: float = 0.0
    http_cpu_ns: int = 0   # the HTTP worker thread(s)
    proc_cpu_ns: int = 0   # the whole exporter process


def _vals(blocks: list, key: str) -> list:
    return [s[key] for b in blocks for s in b.scrapes if s.get(key) is not None]


def _q(v: list, q: float):
    if not v:
        return None
    v = sorted(v)
    k = (len(v) - 1) * q
    lo, hi = int(k), min(int(k) + 1, len(v) - 1)
    return v[lo] + (v[hi] - v[lo]) * (k - lo)


def _cpu_pct(blocks: list, key: str):
    wall = sum(b.wall_s for b in blocks)
    return 100.0 * sum(getattr(b, key) for b in blocks) * 1e-9 / wall if wall > 0 else None


def arm_summary(blocks: list) -> dict:
    n = sum(len(b.scrapes) for b in blocks)
    pw = [s["pw"] for b in blocks for s in b.scrapes if s.get("pw") is not None and s["pw"] >= 0]
    out = {"scrapes": n, "blocks": len(blocks)}
    for name, key in (("total", "total"), ("request_to_server", "req"), ("socket_queue_to_parsed", "sq")):
        v = _vals(blocks, key)
        out[f"{name}_p50_us"] = round(_q(v, 0.5), 2) if v else None
        out[f"{name}_p90_us"] = round(_q(v, 0.9), 2) if v else None
    out["hit_rate"] = round(sum(1 for x in pw if x == 1) / len(pw), 3) if pw else None
    http = sum(b.http_cpu_ns for b in blocks)
    out["http_cpu_us_per_scrape"] = round(http / 1e3 / n, 2) if n else None
    hp, pp = _cpu_pct(blocks, "http_cpu_ns"), _cpu_pct(blocks, "proc_cpu_ns")
    out["http_cpu_percent"] = round(hp, 4) if hp is not None else None
    out["exporter_cpu_percent"] = round(pp, 4) if pp is not None else None
    return out


def bootstrap_diff(a: list, b: list, stat, n_boot: int = 2000, seed: int = 1, alpha: float = 0.05) -> dict:
    """Block bootstrap of stat(b) - stat(a) (lists of Blocks): point estimate and the
    (alpha/2, 1-alpha/2) percentile interval."""
    rng = random.Random(seed)
    point = stat(b) - stat(a)
    d = []
    for _ in range(n_boot):
        ra = [a[rng.randrange(len(a))] for _ in a]
        rb = [b[rng.randrange(len(b))] for _ in b]
        d.append(stat(rb) - stat(ra))
    d.sort()
    return {"diff": round(point, 3), "ci95": [round(d[int(alpha / 2 * n_boot)], 3),
                                              round(d[min(n_boot - 1, int((1 - alpha / 2) * n_boot))], 3)]}


def p50_of(key: str):
    def f(blocks: list) -> float:
        v = _vals(blocks, key)
        return statistics.median(v) if v else float("nan")
    return f


def cpu_of(attr: str):
    def f(blocks: list) -> float:
        v = _cpu_pct(blocks, attr)
        return v if v is not None else float("nan")
    return f


def blocks_to_json(blocks: list) -> list:
    """Raw blocks for re-analysis: [arm, wall_s, http_cpu_ns, proc_cpu_ns, [[total, req, sq, pw], ...]]."""
    return [[b.arm, round(b.wall_s, 6), b.http_cpu_ns, b.proc_cpu_ns,
             [[s.get("total"), s.get("req"), s.get("sq"), s.get("pw")] for s in b.scrapes]] for b in blocks]


def blocks_from_json(raw: list) -> list:
    out = []
    for arm, wall, http, proc, scrapes in raw:
        b = Block(arm, wall_s=wall, http_cpu_ns=http, proc_cpu_ns=proc)
        b.scrapes = [{"total": t, "req": r, "sq": q, "pw": p} for t, r, q, p in scrapes]
        out.append(b)
    return out


def analyse(blocks: list, baseline: str = "off", cpu_budget_pts: float = 0.1, n_boot: int = 2000) -> dict:
    """Per-arm table, bootstrap CIs of every arm against `baseline` (p50 of the total
    latency, of request->server and of socket_queue->parsed; exporter CPU %), and the
    default the data supports, on the combined metric:
      1. an arm qualifies when its p50 CI against the baseline lies wholly below 0 and its
         CPU % is within `cpu_budget_pts` points of the baseline's (point estimate; its CI is
         reported);
      2. the qualifying arm with the lowest p50 leads;
      3. a qualifying arm whose p50 is NOT significantly above the leader's (the CI of the
         difference contains 0) and that costs less CPU replaces it (the cheapest such) --
         latency the data cannot tell apart is not worth CPU.
    No qualifying arm: the baseline."""
    arms = sorted({b.arm for b in blocks}, key=lambda a: (a != baseline, a))
    by = {a: [b for b in blocks if b.arm == a] for a in arms}
    out = {"arms": {a: arm_summary(by[a]) for a in arms}, "baseline": baseline,
           "cpu_budget_points": cpu_budget_pts, "vs_baseline": {}}
    best, best_p50 = baseline, None
    if baseline in by:
        for a in arms:
            if a == baseline:
                continue
            cmp = {"total_p50_us": bootstrap_diff(by[baseline], by[a], p50_of("total"), n_boot),
                   "request_to_server_p50_us": bootstrap_diff(by[baseline], by[a], p50_of("req"), n_boot),
                   "socket_queue_to_parsed_p50_us": bootstrap_diff(by[baseline], by[a], p50_of("sq"), n_boot),
                   "exporter_cpu_points": bootstrap_diff(by[baseline], by[a], cpu_of("proc_cpu_ns"), n_boot),
                   "http_cpu_points": bootstrap_diff(by[baseline], by[a], cpu_of("http_cpu_ns"), n_boot)}
            ok = cmp["total_p50_us"]["ci95"][1] < 0 and cmp["exporter_cpu_points"]["diff"] <= cpu_budget_pts
            cmp["qualifies"] = ok
            out["vs_baseline"][a] = cmp
            p50 = out["arms"][a]["total_p50_us"]
            if ok and (best_p50 is None or p50 < best_p50):
                best, best_p50 = a, p50
    out["leader"] = best
    out["vs_leader"] = {}
    if best != baseline:
        cheapest = best
        for a in arms:
            if a in (baseline, best) or not out["vs_baseline"][a]["qualifies"]:
                continue
            cmp = {"total_p50_us": bootstrap_diff(by[best], by[a], p50_of("total"), n_boot),
                   "exporter_cpu_points": bootstrap_diff(by[best], by[a], cpu_of("proc_cpu_ns"), n_boot)}
            lo, hi = cmp["total_p50_us"]["ci95"]
            cmp["indistinguishable_p50"] = lo <= 0 <= hi
            out["vs_leader"][a] = cmp
            cpu_a = out["arms"][a]["exporter_cpu_percent"]
            if cmp["indistinguishable_p50"] and cpu_a is not None and \
                    cpu_a < out["arms"][cheapest]["exporter_cpu_percent"]:
                cheapest = a
        best = cheapest
    out["chosen_default"] = best
    return out
