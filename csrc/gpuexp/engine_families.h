// Table-driven metric families of the engine, one table per source translation unit:
//
//   engine_device.cc      per-GPU device telemetry (gpu_metrics, counters, sentinel, RAS, ...)
//   engine_procs.cc       per-process families + the reference's two legacy families
//   engine_pods.cc        per-pod aggregates and totals, device-owner inference
//   engine_rccl.cc        RCCL tracer families
//   engine_kfd_events.cc  KFD SMI event families
//   engine_self.cc        gpuexp_* self-observability
//
// A family is one row of its source's FamilySpec table: name, HELP, type, label names and
// how many series handles it keeps (per GPU or global).  Engine::define_families() registers
// every table; an emitter addresses a family by its Fam id and a slot, so adding a family is
// a table row plus the line that sets it (round 5: a definition, a handle member and the
// emitter, in three places of one 2,100-line file).
//
// Reference counterpart: the reference's whole registry is two GaugeVecs
// (/root/reference/main.go:21-42).
#pragma once

#include <cstddef>
#include <string>
#include <vector>

#include "gpuexp/device.h"
#include "gpuexp/exposition.h"
#include "gpuexp/kfd_events.h"

namespace gpuexp {

enum Fam : int {
  // ---- engine_device.cc: per-GPU device families (labels gpu, bdf, namespace, pod, container [+ ...]) ----
  kFamInfo, kFamUp, kFamGfx, kFamUmc, kFamXcc, kFamVramUsed, kFamVramTotal, kFamHbmBw, kFamPower, kFamPowerCap,
  kFamEnergy, kFamTemp, kFamClk, kFamXrd, kFamXwr, kFamXrdRate, kFamXwrRate, kFamLinksUp, kFamPcieBw,
  kFamPcieReplay, kFamPcieSpeed, kFamPcieWidth, kFamThr, kFamNprocs, kFamCuOcc, kFamEcc, kFamAer, kFamPcieNak,
  kFamPcieRecov, kFamXgmiWidth, kFamXgmiSpeed, kFamMfma, kFamMfmaUtil, kFamMfmaFlops, kFamDispStall, kFamOccLim,
  kFamSqBusy, kFamGui, kFamWaves, kFamLds, kFamLdsConf, kFamHbmRd, kFamHbmWr, kFamRemoteRd, kFamRemoteWr,
  kFamSenSclk, kFamSenLat, kFamSenXcc, kFamSenRuns, kFamSenPend, kFamSenMem, kFamXccClk, kFamSenXlat,
  kFamXccMfma, kFamSenXmem, kFamBoard, kFamFw, kFamDriver, kFamPages, kFamGttUsed, kFamGttTotal,
  kFamDevEnd,
  // ---- engine_procs.cc: per-process families ----
  kFamProcVram = kFamDevEnd, kFamProcCu, kFamProcSdma, kFamProcEvicted, kFamProcGfx, kFamLegacyMem,
  kFamLegacyPerc,
  kFamProcEnd,
  // ---- engine_pods.cc: per-pod families ----
  kFamPodVram = kFamProcEnd, kFamPodProcs, kFamPodGpus, kFamPodXrd, kFamPodXwr, kFamPodXrdTotal, kFamPodXwrTotal,
  kFamPodMfma, kFamPodFlops, kFamPodHbm, kFamPodPower, kFamPodAllocS, kFamPodBusyS, kFamPodEnergy, kFamPodGfx,
  kFamPodGfxShare,
  kFamPodEnd,
  // ---- engine_rccl.cc ----
  kFamRcclCalls = kFamPodEnd, kFamRcclBytes, kFamRcclComm, kFamSelfRcclFiles, kFamSelfRcclScans,
  kFamRcclEnd,
  // ---- engine_kfd_events.cc ----
  kFamKfdEv = kFamRcclEnd, kFamPodKfdEv,
  kFamKfdEnd,
  // ---- engine_self.cc: gpuexp_* self-metrics ----
  kFamSelfBuild = kFamKfdEnd, kFamSelfTicks, kFamSelfPodsComplete, kFamSelfKfdScans, kFamSelfKfdTracked,
  kFamSelfStartup, kFamSelfLast, kFamSelfStage, kFamSelfDevPart, kFamSelfFetchCpu, kFamSelfFetchCap,
  kFamSelfMetricsAge, kFamSelfScrape, kFamSelfScrapes, kFamSelfHttpBytes, kFamSelfPrewake, kFamSelfPrewakeHits,
  kFamSelfPrewakeHitsNarrow, kFamSelfPrewakeSpins, kFamSelfPrewakeSpinS, kFamSelfRxMoves, kFamSelfGzip,
  kFamSelfRenderBytes, kFamSelfExpo, kFamSelfSeries, kFamSelfDevErrors, kFamSelfOverruns, kFamSelfCpu,
  kFamSelfSourceUp, kFamSelfMetricsReads, kFamSelfMetricsPeriod, kFamSelfUnresolved, kFamSelfCtrLate,
  kFamSelfCtrEvents, kFamSelfCtrRescue, kFamSelfCtrScope, kFamSelfCtrInterval,
  kFamCount
};

// Label sets a family's names start with; `extra` names follow.
enum class LabelBase : unsigned char {
  kNone,     // only `extra`
  kDevice,   // gpu, bdf, namespace, pod, container
  kProcess,  // gpu, pid, comm, namespace, pod, container
  kPod,      // namespace, pod
};

// Where a family's series handles live: per GPU (DevState::refs, `slots` of them per GPU), in
// the engine's global handle array (`slots`), or keyed by the emitter itself (process, pod, RCCL
// maps: slots unused).
enum class RefScope : unsigned char { kGpu, kGlobal, kKeyed };

struct FamilySpec {
  Fam id;
  const char* name;
  const char* help;
  MetricType type;
  LabelBase base;
  std::vector<const char*> extra;
  RefScope scope;
  int slots;
  bool needs_legacy = false;  // registered only with EngineConfig::legacy_families
};

// The per-source tables (each defined in its own translation unit).
const std::vector<FamilySpec>& device_family_specs();
const std::vector<FamilySpec>& process_family_specs();
const std::vector<FamilySpec>& pod_family_specs();
const std::vector<FamilySpec>& rccl_family_specs();
const std::vector<FamilySpec>& kfd_event_family_specs();
const std::vector<FamilySpec>& self_family_specs();

std::vector<std::string> family_labels(const FamilySpec& s);

}  // namespace gpuexp
