// RAS (ECC) and PCIe AER error totals for one GPU, from sysfs.
//
// The reference exports no health signal at all — a GPU with uncorrectable HBM errors
// keeps reporting memory bytes (/root/reference/main.go:129-150).  amdgpu exposes per-IP
// RAS counters as <pci dev>/ras/<block>_err_count ("ue: N\nce: N[\nde: N]") and the PCI
// core exposes AER totals as <pci dev>/aer_dev_{correctable,nonfatal,fatal}
// ("... TOTAL_ERR_COR N").  A RAS query can reach the PSP firmware, so the engine reads
// these at a low rate (EngineConfig::ras_interval_s) and keeps the last totals between
// reads.  Everything here is plain file IO under an injectable host root.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "gpuexp/device.h"

namespace gpuexp {

struct RasTotals {
  double ecc_ce = kNaN, ecc_ue = kNaN, ecc_de = kNaN;
  double aer_cor = kNaN, aer_nonfatal = kNaN, aer_fatal = kNaN;
  // HBM pages in the RAS bad-page table (ras/gpu_vram_bad_pages): retired (reserved, never
  // handed out again), pending retirement, and ones the driver could not reserve
  double pages_retired = kNaN, pages_pending = kNaN, pages_unreservable = kNaN;
};

// Parses one amdgpu ras/<block>_err_count body; adds into *t (NaN fields start at 0).
bool parse_ras_err_count(const std::string& body, RasTotals* t);
// Parses one aer_dev_* body; returns the TOTAL_ERR_* value or NaN.
double parse_aer_total(const std::string& body);
// Parses ras/gpu_vram_bad_pages ("0x<page> : 0x<size> : R|P|F" per page); sets the three
// page counts of *t.  False when no line parses (and the body is not empty).
bool parse_bad_pages(const std::string& body, RasTotals* t);

class RasReader {
 public:
  // pci_dev_dir: <root>/sys/bus/pci/devices/<bdf>
  void open(const std::string& pci_dev_dir);
  // Re-reads every file; returns false when the device exposes neither RAS nor AER.
  bool read(RasTotals* out) const;
  size_t files() const { return ras_files_.size() + (aer_dir_.empty() ? 0 : 3) + (bad_pages_.empty() ? 0 : 1); }

 private:
  std::vector<std::string> ras_files_;
  std::string aer_dir_;
  std::string bad_pages_;
};

}  // namespace gpuexp
