// kaldi-lite/kaldi-common.h -- the slice of Kaldi's base/ the plugin uses
// (SURVEY Appendix C): integer/float typedefs, resize/transpose enums and the
// KALDI_ASSERT / KALDI_ERR / KALDI_WARN / KALDI_LOG macros.
//
// Error behaviour: like upstream Kaldi, KALDI_ERR throws.  KALDI_ASSERT throws
// too (upstream aborts) so that the extern "C" boundary can turn it into an
// error code instead of killing a host process that embeds the library.
#ifndef KCNN_KALDI_LITE_KALDI_COMMON_H_
#define KCNN_KALDI_LITE_KALDI_COMMON_H_

#include <stdint.h>

#include <sstream>
#include <stdexcept>
#include <string>

namespace kaldi {

typedef int32_t int32;
typedef int64_t int64;
typedef uint32_t uint32;
typedef float BaseFloat;
typedef int32 MatrixIndexT;

enum MatrixResizeType { kSetZero, kUndefined, kCopyData };
// Values of CBLAS_TRANSPOSE, as in Kaldi's matrix-common.h.
enum MatrixTransposeType { kTrans = 112, kNoTrans = 111 };

class KaldiFatalError : public std::runtime_error {
 public:
  explicit KaldiFatalError(const std::string &msg) : std::runtime_error(msg) {}
};

int GetVerboseLevel();
void SetVerboseLevel(int v);

// Stream that throws (ERROR) or prints (WARNING/LOG) at the end of the
// full-expression, like Kaldi's MessageLogger.
class MessageLogger {
 public:
  enum Severity { kError = -2, kWarning = -1, kInfo = 0 };
  MessageLogger(Severity sev, const char *func, const char *file, int line);
  ~MessageLogger() noexcept(false);
  std::ostream &stream() { return ss_; }

 private:
  Severity sev_;
  std::ostringstream ss_;
};

[[noreturn]] void KaldiAssertFailure(const char *func, const char *file,
                                     int line, const char *cond);

}  // namespace kaldi

#define KALDI_ERR                                                       \
  ::kaldi::MessageLogger(::kaldi::MessageLogger::kError, __func__, __FILE__, \
                         __LINE__)                                     \
      .stream()
#define KALDI_WARN                                                        \
  ::kaldi::MessageLogger(::kaldi::MessageLogger::kWarning, __func__, __FILE__, \
                         __LINE__)                                       \
      .stream()
#define KALDI_LOG                                                      \
  ::kaldi::MessageLogger(::kaldi::MessageLogger::kInfo, __func__, __FILE__, \
                         __LINE__)                                    \
      .stream()
#define KALDI_ASSERT(cond)                                                 \
  do {                                                                     \
    if (!(cond)) ::kaldi::KaldiAssertFailure(__func__, __FILE__, __LINE__, \
                                             #cond);                       \
  } while (0)

#define KALDI_DISALLOW_COPY_AND_ASSIGN(type) \
  type(const type &) = delete;               \
  void operator=(const type &) = delete

#endif  // KCNN_KALDI_LITE_KALDI_COMMON_H_
