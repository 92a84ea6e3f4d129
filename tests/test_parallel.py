"""Traffic generators for every parallelism strategy, on CPU with gloo (world_size 2 and 4):
results are checked inside the workers; the per-rank byte accounting must match the RCCL
tracer's formulas (what the exporter reports per pod)."""
import pytest

from kubernetes_gpu_exporter_amd.parallel.collectives import STRATEGIES, ring_allreduce_link_bytes
from kubernetes_gpu_exporter_amd.parallel.launch import spawn, traffic_worker

NB = 4096  # bytes per message (float32: 1024 elements)


@pytest.mark.parametrize("strategy", STRATEGIES)
def test_strategy_world2(strategy):
    res = spawn(traffic_worker, 2, "gloo", args=(strategy, 2, NB))
    r0, r1 = res
    if strategy == "dp":
        assert r0["calls"] == {"allreduce": 2} and r0["bytes"]["allreduce"] == 2 * NB
    elif strategy == "tp":
        assert r0["calls"] == {"allreduce": 4, "allgather": 4}
    elif strategy == "sp":
        assert r0["bytes"] == {"allgather": 2 * NB, "reducescatter": 2 * NB}
    elif strategy == "ep":
        assert r0["calls"] == {"alltoall": 2} and r0["bytes"]["alltoall"] == 2 * NB
    elif strategy == "ulysses":
        assert r0["calls"] == {"alltoall": 8}
    elif strategy == "pp":
        assert r0["calls"] == {"send": 2} and r1["calls"] == {"recv": 2}  # asymmetric by stage
    elif strategy == "cp":
        assert r0["calls"] == {"send": 2, "recv": 2} == r1["calls"]  # ring: both neighbours
    elif strategy == "bcast":
        assert r0["calls"] == {"broadcast": 2, "reduce": 2} == r1["calls"]
        assert r0["bytes"] == {"broadcast": 2 * NB, "reduce": 2 * NB}


def test_strategies_world4():
    res = spawn(traffic_worker, 4, "gloo", args=("cp", 1, NB))
    assert all(r["calls"] == {"send": 3, "recv": 3} for r in res)  # world-1 hops
    res = spawn(traffic_worker, 4, "gloo", args=("pp", 1, NB))
    assert [sorted(r["calls"]) for r in res] == [["send"], ["recv", "send"], ["recv", "send"], ["recv"]]


def test_ring_model():
    assert ring_allreduce_link_bytes(1 << 20, 1) == 0
    assert ring_allreduce_link_bytes(800, 8) == 1400
