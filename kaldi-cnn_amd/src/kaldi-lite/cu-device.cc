// kaldi-lite/cu-device.cc
#include "cu-device.h"

#include <stdio.h>
#include <stdlib.h>

#include <iomanip>
#include <iostream>

namespace kaldi {

static int g_verbose = 0;
int GetVerboseLevel() { return g_verbose; }
void SetVerboseLevel(int v) { g_verbose = v; }

MessageLogger::MessageLogger(Severity sev, const char *func, const char *file,
                             int line)
    : sev_(sev) {
  const char *base = file;
  for (const char *p = file; *p; ++p)
    if (*p == '/') base = p + 1;
  const char *tag = sev == kError ? "ERROR" : sev == kWarning ? "WARNING" : "LOG";
  ss_ << tag << " (" << func << "():" << base << ":" << line << ") ";
}

MessageLogger::~MessageLogger() noexcept(false) {
  if (sev_ == kError) throw KaldiFatalError(ss_.str());
  if (sev_ == kWarning || g_verbose >= 0) {
    if (sev_ == kInfo && getenv("KCNN_QUIET")) return;
    std::cerr << ss_.str() << std::endl;
  }
}

void KaldiAssertFailure(const char *func, const char *file, int line,
                        const char *cond) {
  std::ostringstream ss;
  const char *base = file;
  for (const char *p = file; *p; ++p)
    if (*p == '/') base = p + 1;
  ss << "ASSERTION_FAILED (" << func << "():" << base << ":" << line << ") "
     << cond;
  throw KaldiFatalError(ss.str());
}

// ---------------------------------------------------------------------------
namespace {
struct PendingEvent {
  std::string key;
  hipEvent_t beg, end;
};
std::vector<PendingEvent> &pending() {
  static std::vector<PendingEvent> p;
  return p;
}
// guards pending(), event_pool() and the profile map: profiled scopes may
// close on several host threads at once
std::mutex &prof_mu() {
  static std::mutex m;
  return m;
}
// Events of resolved scopes are kept for reuse: a profiled step creates no
// new events once the pool holds one pair per scope.
std::vector<hipEvent_t> &event_pool() {
  static std::vector<hipEvent_t> p;
  return p;
}
hipEvent_t take_event() {
  std::lock_guard<std::mutex> lk(prof_mu());
  auto &p = event_pool();
  if (!p.empty()) {
    hipEvent_t e = p.back();
    p.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  return hipEventCreate(&e) == hipSuccess ? e : nullptr;
}
void give_event_locked(hipEvent_t e) {
  if (e) event_pool().push_back(e);
}
void give_event(hipEvent_t e) {
  std::lock_guard<std::mutex> lk(prof_mu());
  give_event_locked(e);
}
size_t round_block(size_t bytes) {
  // 256-B granules below 1 MiB, 1 MiB granules above: bounded waste, high reuse.
  if (bytes < (1u << 20)) return (bytes + 255) & ~(size_t)255;
  return (bytes + (1u << 20) - 1) & ~(size_t)((1u << 20) - 1);
}
}  // namespace

CuDevice &CuDevice::Instantiate() {
  static CuDevice *dev = new CuDevice();  // never destroyed (atexit ordering)
  return *dev;
}

CuDevice::CuDevice() {
  if (getenv("KCNN_PROFILE")) profiling_ = atoi(getenv("KCNN_PROFILE")) != 0;
}
CuDevice::~CuDevice() {}

void CuDevice::SelectGpuId(const std::string &use_gpu, int device_id) {
  if (use_gpu == "no")
    KALDI_ERR << "this build has no CPU path: --use-gpu=no is not supported "
                 "(the CPU reference lives in oracle/, as a test checker)";
  int count = 0;
  CU_SAFE_CALL(hipGetDeviceCount(&count));
  if (count <= 0) KALDI_ERR << "no HIP device available";
  if (device_id < 0) CU_SAFE_CALL(hipGetDevice(&device_id));
  if (device_id >= count) KALDI_ERR << "device " << device_id << " >= " << count;
  CU_SAFE_CALL(hipSetDevice(device_id));
  if (active_device_ != device_id) {
    active_device_ = device_id;
    if (blas_) { rocblas_destroy_handle(blas_); blas_ = nullptr; }
  }
  EnsureInit();
}

void CuDevice::EnsureInit() {
  if (active_device_ < 0) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
      KALDI_ERR << "no HIP device available (the product path is GPU-only)";
    int dev = 0;
    CU_SAFE_CALL(hipGetDevice(&dev));
    active_device_ = dev;
  }
  if (!blas_) {
    if (rocblas_create_handle(&blas_) != rocblas_status_success)
      KALDI_ERR << "rocblas_create_handle failed";
    // Deterministic GEMMs (no atomic split-K reductions).
    rocblas_set_atomics_mode(blas_, rocblas_atomics_not_allowed);
    rocblas_set_pointer_mode(blas_, rocblas_pointer_mode_host);
    rocblas_set_stream(blas_, stream_);
  }
}

void CuDevice::SetStream(hipStream_t s) {
  EnsureInit();
  // Cached blocks and the workspace are reused in stream order on stream_:
  // let the old stream drain before kernels on the new one can get them.
  if (s != stream_) CU_SAFE_CALL(hipStreamSynchronize(stream_));
  stream_ = s;
  rocblas_set_stream(blas_, stream_);
}

uint64_t CuDevice::MallocCalls() {
  std::lock_guard<std::mutex> lk(mu_);
  return malloc_calls_;
}

void *CuDevice::Malloc(size_t bytes) {
  EnsureInit();
  if (bytes == 0) bytes = 1;
  const size_t sz = round_block(bytes);
  std::lock_guard<std::mutex> lk(mu_);
  ++malloc_calls_;
  auto it = free_blocks_.find(sz);
  void *p = nullptr;
  if (it != free_blocks_.end()) {
    p = it->second;
    free_blocks_.erase(it);
    bytes_cached_ -= sz;
  } else {
    hipError_t e = hipMalloc(&p, sz);
    if (e != hipSuccess) {
      // Give the cache back and retry once.
      for (auto &kv : free_blocks_) (void)hipFree(kv.second);
      free_blocks_.clear();
      bytes_cached_ = 0;
      e = hipMalloc(&p, sz);
      if (e != hipSuccess)
        KALDI_ERR << "hipMalloc(" << sz << ") failed: " << hipGetErrorString(e);
    }
  }
  live_blocks_[p] = sz;
  bytes_in_use_ += sz;
  return p;
}

void CuDevice::Free(void *ptr) {
  if (!ptr) return;
  std::lock_guard<std::mutex> lk(mu_);
  auto it = live_blocks_.find(ptr);
  if (it == live_blocks_.end()) KALDI_ERR << "CuDevice::Free of unknown pointer";
  const size_t sz = it->second;
  live_blocks_.erase(it);
  bytes_in_use_ -= sz;
  // Stream-ordered reuse: every user of the block ran on stream_, so a later
  // allocation's kernels on stream_ cannot overtake the earlier uses.
  free_blocks_.emplace(sz, ptr);
  bytes_cached_ += sz;
}

void CuDevice::ReleaseCache() {
  Synchronize();
  std::lock_guard<std::mutex> lk(mu_);
  for (auto &kv : free_blocks_) (void)hipFree(kv.second);
  free_blocks_.clear();
  bytes_cached_ = 0;
}

void CuDevice::Synchronize() {
  EnsureInit();
  CU_SAFE_CALL(hipStreamSynchronize(stream_));
}

void CuDevice::AccuProfile(const std::string &key, double ms) {
  std::lock_guard<std::mutex> lk(prof_mu());
  AccuProfileLocked(key, ms);
}

void CuDevice::AccuProfileLocked(const std::string &key, double ms) {
  auto &e = profile_[key];
  e.first += ms;
  e.second += 1;
}

std::string CuDevice::ProfileString() const {
  CuDevice *self = const_cast<CuDevice *>(this);
  std::lock_guard<std::mutex> lk(prof_mu());
  for (auto &pe : pending()) {
    float ms = 0.0f;
    if (hipEventSynchronize(pe.end) == hipSuccess &&
        hipEventElapsedTime(&ms, pe.beg, pe.end) == hipSuccess)
      self->AccuProfileLocked(pe.key, ms);
    give_event_locked(pe.beg);
    give_event_locked(pe.end);
  }
  pending().clear();
  std::ostringstream os;
  os << std::fixed << std::setprecision(4);
  for (auto &kv : profile_)
    os << kv.first << "\t" << kv.second.first << " ms\t" << kv.second.second
       << " calls\n";
  return os.str();
}

CuProfileScope::CuProfileScope(const char *key) : key_(key) {
  CuDevice &d = CuDevice::Instantiate();
  if (!d.Profiling()) return;
  beg_ = take_event();
  end_ = take_event();
  if (!beg_ || !end_) {
    give_event(beg_);
    give_event(end_);
    beg_ = end_ = nullptr;
    return;
  }
  (void)hipEventRecord(beg_, d.Stream());
}

void CuProfileScope::Cancel() {
  if (!beg_) return;
  give_event(beg_);
  give_event(end_);
  beg_ = end_ = nullptr;
}

CuProfileScope::~CuProfileScope() {
  if (!beg_) return;
  CuDevice &d = CuDevice::Instantiate();
  (void)hipEventRecord(end_, d.Stream());
  std::lock_guard<std::mutex> lk(prof_mu());
  pending().push_back({key_, beg_, end_});
}

}  // namespace kaldi
