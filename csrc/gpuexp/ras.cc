#include "gpuexp/ras.h"

#include <unistd.h>

#include <cmath>
#include <cstdlib>

#include "gpuexp/common.h"

namespace gpuexp {

namespace {

void add(double* field, double v) { *field = (std::isnan(*field) ? 0.0 : *field) + v; }

bool parse_num(const std::string& s, uint64_t* v) { return parse_u64(s.data(), s.size(), v); }

}  // namespace

bool parse_ras_err_count(const std::string& body, RasTotals* t) {
  bool any = false;
  size_t pos = 0;
  while (pos < body.size()) {
    size_t eol = body.find('\n', pos);
    if (eol == std::string::npos) eol = body.size();
    const std::string line = trim(body.substr(pos, eol - pos));
    pos = eol + 1;
    const size_t colon = line.find(':');
    if (colon == std::string::npos) continue;
    const std::string key = trim(line.substr(0, colon));
    uint64_t v = 0;
    if (!parse_num(trim(line.substr(colon + 1)), &v)) continue;
    if (key == "ue") add(&t->ecc_ue, double(v)), any = true;
    else if (key == "ce") add(&t->ecc_ce, double(v)), any = true;
    else if (key == "de") add(&t->ecc_de, double(v)), any = true;
  }
  return any;
}

double parse_aer_total(const std::string& body) {
  size_t p = body.find("TOTAL_ERR_");
  if (p == std::string::npos) return kNaN;
  p = body.find_first_of(" \t", p);
  if (p == std::string::npos) return kNaN;
  size_t e = body.find('\n', p);
  uint64_t v = 0;
  if (!parse_num(trim(body.substr(p, e == std::string::npos ? std::string::npos : e - p)), &v)) return kNaN;
  return double(v);
}

bool parse_bad_pages(const std::string& body, RasTotals* t) {
  double r = 0, p = 0, f = 0;
  bool any = false, bad = false;
  size_t pos = 0;
  while (pos < body.size()) {
    size_t eol = body.find('\n', pos);
    if (eol == std::string::npos) eol = body.size();
    const std::string line = trim(body.substr(pos, eol - pos));
    pos = eol + 1;
    if (line.empty()) continue;
    const size_t c = line.rfind(':');
    const std::string st = c == std::string::npos ? std::string() : trim(line.substr(c + 1));
    if (st == "R") r += 1;
    else if (st == "P") p += 1;
    else if (st == "F") f += 1;
    else {
      bad = true;
      continue;
    }
    any = true;
  }
  if (bad && !any) return false;
  t->pages_retired = r;
  t->pages_pending = p;
  t->pages_unreservable = f;
  return true;
}

void RasReader::open(const std::string& pci_dev_dir) {
  ras_files_.clear();
  aer_dir_.clear();
  bad_pages_.clear();
  if (::access((pci_dev_dir + "/ras/gpu_vram_bad_pages").c_str(), R_OK) == 0)
    bad_pages_ = pci_dev_dir + "/ras/gpu_vram_bad_pages";
  const std::string ras = pci_dev_dir + "/ras";
  for (const auto& f : list_dir(ras)) {
    const std::string suffix = "_err_count";
    if (f.size() > suffix.size() && f.compare(f.size() - suffix.size(), suffix.size(), suffix) == 0)
      ras_files_.push_back(ras + "/" + f);
  }
  if (::access((pci_dev_dir + "/aer_dev_correctable").c_str(), R_OK) == 0) aer_dir_ = pci_dev_dir;
}

bool RasReader::read(RasTotals* out) const {
  RasTotals t;
  bool any = false;
  std::string body;
  for (const auto& f : ras_files_)
    if (read_small_file(f, &body)) any |= parse_ras_err_count(body, &t);
  if (!bad_pages_.empty() && read_small_file(bad_pages_, &body, 1 << 20)) any |= parse_bad_pages(body, &t);
  if (!aer_dir_.empty()) {
    if (read_small_file(aer_dir_ + "/aer_dev_correctable", &body)) t.aer_cor = parse_aer_total(body);
    if (read_small_file(aer_dir_ + "/aer_dev_nonfatal", &body)) t.aer_nonfatal = parse_aer_total(body);
    if (read_small_file(aer_dir_ + "/aer_dev_fatal", &body)) t.aer_fatal = parse_aer_total(body);
    any = true;
  }
  *out = t;
  return any;
}

}  // namespace gpuexp
