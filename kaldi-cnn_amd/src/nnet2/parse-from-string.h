// nnet2/parse-from-string.h -- "name=value" option parsers used by the
// components' InitFromString (reference nnet-component-nnet0.cc:42-176):
// on a match the option is removed from *string and true is returned; a
// malformed value is a KALDI_ERR.
#ifndef KCNN_NNET2_PARSE_FROM_STRING_H_
#define KCNN_NNET2_PARSE_FROM_STRING_H_

#include <string>
#include <vector>

#include "../kaldi-lite/kaldi-common.h"

namespace kaldi {
namespace nnet2 {
bool ParseFromString(const std::string &name, std::string *string, int32 *param);
bool ParseFromString(const std::string &name, std::string *string, bool *param);
bool ParseFromString(const std::string &name, std::string *string, BaseFloat *param);
bool ParseFromString(const std::string &name, std::string *string, std::string *param);
bool ParseFromString(const std::string &name, std::string *string,
                     std::vector<int32> *param);
}  // namespace nnet2
}  // namespace kaldi

#endif
