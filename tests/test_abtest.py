"""The in-process A/B analysis behind bench.py --prewake-ab (utils/abtest.py): block order,
block bootstrap, and the default it picks."""
import random

from kubernetes_gpu_exporter_amd.utils import abtest


def test_block_schedule_rounds_are_permutations():
    s = abtest.block_schedule(["off", "slices", "spin"], 30, seed=4)
    assert len(s) == 30
    for r in range(10):
        assert sorted(s[3 * r:3 * r + 3]) == ["off", "slices", "spin"]
    assert s != abtest.block_schedule(["off", "slices", "spin"], 30, seed=5)
    assert abtest.block_schedule(["a", "b"], 3, seed=1)[:2] in (["a", "b"], ["b", "a"])


def _blocks(arm, p50, cpu_ns, n_blocks=30, per=10, seed=0, sd=5.0):
    rng = random.Random(seed)
    out = []
    for _ in range(n_blocks):
        b = abtest.Block(arm)
        for _ in range(per):
            v = rng.gauss(p50, sd)
            b.scrapes.append({"total": v, "req": v / 2, "sq": v / 4, "pw": 1 if arm != "off" else 0})
        b.wall_s = 1.0
        b.http_cpu_ns = b.proc_cpu_ns = int(cpu_ns + rng.gauss(0, cpu_ns * 0.05))
        out.append(b)
    return out


def test_analyse_picks_the_faster_arm_within_the_cpu_budget():
    # 1 s blocks: 5 ms of CPU = 0.5 %
    blocks = _blocks("off", 100, 5_000_000, seed=1) + _blocks("spin", 60, 5_500_000, seed=2) + \
        _blocks("slices", 80, 5_200_000, seed=3)
    r = abtest.analyse(blocks, n_boot=400)
    assert r["chosen_default"] == "spin"
    v = r["vs_baseline"]["spin"]
    lo, hi = v["total_p50_us"]["ci95"]
    assert lo <= -40 + 5 and hi < 0 and v["qualifies"]
    assert abs(v["exporter_cpu_points"]["diff"] - 0.05) < 0.03
    a = r["arms"]["spin"]
    assert a["scrapes"] == 300 and a["hit_rate"] == 1.0 and abs(a["total_p50_us"] - 60) < 2


def test_analyse_keeps_the_baseline_without_evidence_or_over_budget():
    # no difference in p50: the CI straddles 0
    blocks = _blocks("off", 100, 5_000_000, seed=1) + _blocks("spin", 100, 5_000_000, seed=2)
    assert abtest.analyse(blocks, n_boot=400)["chosen_default"] == "off"
    # faster but +0.5 points of CPU (budget 0.1)
    blocks = _blocks("off", 100, 5_000_000, seed=1) + _blocks("spin", 50, 10_000_000, seed=2)
    r = abtest.analyse(blocks, n_boot=400)
    assert r["chosen_default"] == "off" and not r["vs_baseline"]["spin"]["qualifies"]


def test_analyse_prefers_the_cheaper_of_two_indistinguishable_arms():
    # both beat the baseline; spin is 2 us faster (not resolvable at sd 5 with these blocks)
    # but costs more CPU: the cheaper arm is chosen
    blocks = _blocks("off", 100, 5_000_000, seed=1) + _blocks("spin", 58, 5_800_000, seed=2, sd=15) + \
        _blocks("slices", 60, 5_200_000, seed=3, sd=15)
    r = abtest.analyse(blocks, n_boot=400)
    assert r["leader"] == "spin" and r["vs_leader"]["slices"]["indistinguishable_p50"]
    assert r["chosen_default"] == "slices"


def test_blocks_round_trip_through_json():
    import json
    blocks = _blocks("off", 100, 5_000_000, n_blocks=3) + _blocks("spin", 60, 5_500_000, n_blocks=3)
    back = abtest.blocks_from_json(json.loads(json.dumps(abtest.blocks_to_json(blocks))))
    assert [b.arm for b in back] == [b.arm for b in blocks]
    assert abtest.analyse(back, n_boot=100)["arms"] == abtest.analyse(blocks, n_boot=100)["arms"]
