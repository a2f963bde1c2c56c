// kaldi-lite/kcnn-knobs.cc -- see kcnn-knobs.h.
#include "kcnn-knobs.h"

#include <stdlib.h>
#include <string.h>

#include <atomic>

namespace kcnn {
namespace {

struct FamilyInfo {
  const char *name, *env;
  int dflt, max;
};
const FamilyInfo kFamilies[kNumFamilies] = {
    {"fwd_x6", "KCNN_FWD_X6", 2, 2},
    {"bwd_x6", "KCNN_BWD_X6", 1, 1},
    {"igemm_x6", "KCNN_IGEMM_X6", 2, 3},
    {"wgrad_x6", "KCNN_WGRAD_X6", 2, 3},
    {"gemm", "KCNN_GEMM", 2, 2},
};

int from_env(const FamilyInfo &f) {
  const char *e = getenv(f.env);
  if (!e || !*e) return f.dflt;
  const int v = atoi(e);
  return v < 0 ? 0 : v > f.max ? f.max : v;
}

std::atomic<int> *values() {
  static std::atomic<int> v[kNumFamilies];
  static const bool init = [] {
    for (int i = 0; i < kNumFamilies; ++i) v[i].store(from_env(kFamilies[i]));
    return true;
  }();
  (void)init;
  return v;
}

}  // namespace

int family(Family f) { return values()[f].load(std::memory_order_relaxed); }

int set_family(Family f, int value) {
  if (f < 0 || f >= kNumFamilies || value < 0 || value > kFamilies[f].max) return -1;
  values()[f].store(value);
  return 0;
}

int family_by_name(const char *name) {
  if (!name) return -1;
  for (int i = 0; i < kNumFamilies; ++i)
    if (strcmp(name, kFamilies[i].name) == 0) return i;
  return -1;
}

int experiment_env(const char *name, int dflt) {
  const char *s = getenv(name);
  return s && *s ? atoi(s) : dflt;
}

}  // namespace kcnn
