"""The device-counter derivations both PMC plugins share (csrc/gpuexp/counter_model.h),
on hand-made counter deltas: formulas, units and the scope rule.  On-silicon calibration of
the same outputs: tests/test_gpu.py::test_device_scope_pmc_calibration and the MFMA ones."""
import math

import pytest

SIMD, CU = 1024, 256  # MI355X: 256 CUs x 4 SIMDs
# output order: counter_model.h derive() / optional_sources.cc sample()
(MFMA_BUSY, SQ_BUSY, GUI, WAVES, LDS, LDS_CONF, HBM_RD, HBM_WR, GMI_RD, GMI_WR, MFMA_UTIL, BF16, FP8,
 STALL, LIM_LDS, LIM_WAVES, LIM_VGPR, LIM_SGPR) = range(18)


def derive(native, wall=0.1, privileged=True, **deltas):
    return native.derive_counters(deltas, wall, SIMD, CU, privileged)


def test_mfma_busy_and_util(native):
    clk = 2.0e8  # 100 ms at 2 GHz
    out, _ = derive(native, GRBM_COUNT=clk, GRBM_GUI_ACTIVE=clk / 2, SQ_VALU_MFMA_BUSY_CYCLES=0.25 * clk * SIMD)
    assert out[MFMA_BUSY] == pytest.approx(25.0)   # over elapsed cycles
    assert out[MFMA_UTIL] == pytest.approx(50.0)   # over GUI-active cycles (MfmaUtil)
    assert out[GUI] == pytest.approx(50.0)


def test_bandwidth_and_flops_units(native):
    out, _ = derive(native, wall=0.5, TCC_EA0_RDREQ_DRAM_32B=1e9, TCC_EA0_WRREQ_WRITE_DRAM_32B=5e8,
                    TCC_EA0_RDREQ_GMI_32B=2e6, SQ_INSTS_VALU_MFMA_MOPS_BF16=1e12, SQ_INSTS_VALU_MFMA_MOPS_F8=3e11,
                    SQ_WAVES=4e5, GRBM_COUNT=1e8, GRBM_GUI_ACTIVE=1e8)
    assert out[HBM_RD] == pytest.approx(1e9 * 32 / 0.5)        # 32-B sectors
    assert out[HBM_WR] == pytest.approx(5e8 * 32 / 0.5)
    assert out[GMI_RD] == pytest.approx(2e6 * 32 / 0.5)
    assert out[BF16] == pytest.approx(1e12 * 512 / 0.5)        # MOPS x 512 FLOPs
    assert out[FP8] == pytest.approx(3e11 * 512 / 0.5)
    assert out[WAVES] == pytest.approx(4e5 / 0.5)


def test_lds_ratios(native):
    out, _ = derive(native, GRBM_COUNT=1e8, GRBM_GUI_ACTIVE=1e8, SQ_LDS_IDX_ACTIVE=0.1 * 1e8 * CU,
                    SQ_LDS_BANK_CONFLICT=0.1 * 1e8 * CU * 31 / 32)
    assert out[LDS] == pytest.approx(10.0)
    assert out[LDS_CONF] == pytest.approx(100 * 31 / 32)
    idle, _ = derive(native, GRBM_COUNT=1e8)
    assert idle[LDS_CONF] == 0.0 and math.isnan(idle[LDS])  # no GUI-active cycles: no LDS share


def test_scope_follows_privilege(native):
    _, scope = derive(native, privileged=False, GRBM_COUNT=1e8, GRBM_GUI_ACTIVE=1e8)
    assert scope == 0  # unprivileged: wave / LDS / EA / MOPS counters are VMID-filtered
    _, scope = derive(native, privileged=True, GRBM_COUNT=1e8, GRBM_GUI_ACTIVE=1e8, SQ_WAVES=1e6)
    assert scope == 1
    # privileged but a busy MFMA window with (almost) no waves: the filter is on after all
    _, scope = derive(native, privileged=True, GRBM_COUNT=1e8, GRBM_GUI_ACTIVE=1e8,
                      SQ_VALU_MFMA_BUSY_CYCLES=1e10, SQ_WAVES=10)
    assert scope == 0


def test_unknown_counter_is_rejected(native):
    with pytest.raises(ValueError):
        derive(native, NOT_A_COUNTER=1)


def test_occupancy_limiters(native):
    """SPI resource-allocator counters: the stall share is over elapsed cycles (per SE); each
    limiter is the share of the SE's CUs (LDS) or SIMDs (wave slots, VGPRs, SGPRs) that were full
    over the stalled cycles.  (derive_counters passes each counter as one instance, i.e. one
    SE holding all CUs.)"""
    clk = 2.0e8
    # the allocator arbitrates every 4th clock: 0.1 x clk stalled arbitration cycles = 40 %
    out, _ = derive(native, GRBM_COUNT=clk, GRBM_GUI_ACTIVE=clk, SPI_RA_RES_STALL_CSN=0.1 * clk,
                    SPI_RA_LDS_CU_FULL_CSN=0.1 * clk * CU * 0.9, SPI_RA_WAVE_SIMD_FULL_CSN=0.1 * clk * SIMD * 0.05,
                    SPI_RA_VGPR_SIMD_FULL_CSN=0, SPI_RA_SGPR_SIMD_FULL_CSN=0.1 * clk * SIMD * 0.25)
    assert out[STALL] == pytest.approx(40.0)
    assert out[LIM_LDS] == pytest.approx(90.0)
    assert out[LIM_WAVES] == pytest.approx(5.0)
    assert out[LIM_VGPR] == 0.0
    assert out[LIM_SGPR] == pytest.approx(25.0)
    idle, _ = derive(native, GRBM_COUNT=clk, GRBM_GUI_ACTIVE=clk, SPI_RA_RES_STALL_CSN=0, SPI_RA_LDS_CU_FULL_CSN=0,
                     SPI_RA_WAVE_SIMD_FULL_CSN=0, SPI_RA_VGPR_SIMD_FULL_CSN=0)
    assert idle[STALL] == 0.0 and idle[LIM_LDS] == 0.0 and idle[LIM_WAVES] == 0.0  # nothing waited
    none, _ = derive(native, GRBM_COUNT=clk, GRBM_GUI_ACTIVE=clk)  # no SPI counters programmed
    assert math.isnan(none[STALL]) and math.isnan(none[LIM_LDS])


def _deltas(native, grbm=2e8, **kw):
    names = native.counter_names()
    d = [0.0] * len(names)
    d[names.index("GRBM_COUNT")] = grbm
    for k, v in kw.items():
        d[names.index(k)] = v
    return d


def test_window_action_rearms_after_a_foreign_reset_or_stop(native):
    """Continuous counting's per-window decision (aql_pmc.cc read_round): a counter that went
    backwards (another profiler's start packet reset / re-programmed them) re-arms at once;
    GRBM_COUNT standing still over real time (someone stopped counting) re-arms on the second
    such window; the first window after arming is skipped (no previous read)."""
    act = native.counter_window_action
    assert act(_deltas(native), True, 0.1) == ("skip", 0)
    assert act(_deltas(native), False, 0.1) == ("publish", 0)
    back = _deltas(native, SQ_WAVES=-5.0)
    assert act(back, False, 0.1) == ("rearm", 0)
    stopped = _deltas(native, grbm=0.0)
    a1, z1 = act(stopped, False, 0.1)
    assert (a1, z1) == ("publish", 1)  # one fluke: still exported (all-zero window)
    assert act(stopped, False, 0.1, z1) == ("rearm", 0)  # the second in a row: re-arm
    assert act(_deltas(native), False, 0.1, 1) == ("publish", 0)  # a moving window clears the streak
    assert act(stopped, False, 0.001, 1) == ("publish", 0)  # too short to tell: no streak
