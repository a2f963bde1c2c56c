// kaldi-lite/kaldi-io.h -- Kaldi's token / basic-type stream I/O (upstream
// base/io-funcs.h) and the text helpers of util/text-utils.h that the
// component parsers use.  Binary and text encodings follow upstream Kaldi:
// tokens are followed by one space; binary basic types are a size byte then
// the raw little-endian value; bool is 'T'/'F'.
#ifndef KCNN_KALDI_LITE_KALDI_IO_H_
#define KCNN_KALDI_LITE_KALDI_IO_H_

#include <istream>
#include <ostream>
#include <string>
#include <vector>

#include "kaldi-common.h"

namespace kaldi {

void WriteToken(std::ostream &os, bool binary, const std::string &token);
void ReadToken(std::istream &is, bool binary, std::string *token);
void ExpectToken(std::istream &is, bool binary, const std::string &token);
int PeekToken(std::istream &is, bool binary);

void WriteBasicType(std::ostream &os, bool binary, int32 t);
void WriteBasicType(std::ostream &os, bool binary, float t);
void WriteBasicType(std::ostream &os, bool binary, bool t);
void ReadBasicType(std::istream &is, bool binary, int32 *t);
void ReadBasicType(std::istream &is, bool binary, float *t);
void ReadBasicType(std::istream &is, bool binary, bool *t);
void WriteBasicType(std::ostream &os, bool binary, double t);
void ReadBasicType(std::istream &is, bool binary, double *t);
// upstream base/io-funcs-inl.h WriteIntegerVector / ReadIntegerVector (int32):
// binary = size byte, int32 count, raw values; text = "[ v1 v2 ... ]".
void WriteIntegerVector(std::ostream &os, bool binary, const std::vector<int32> &v);
void ReadIntegerVector(std::istream &is, bool binary, std::vector<int32> *v);

// Kaldi binary-mode header "\0B" (util/kaldi-io.cc InitKaldiInputStream).
void InitKaldiOutputStream(std::ostream &os, bool binary);
bool InitKaldiInputStream(std::istream &is, bool *binary);

void SplitStringToVector(const std::string &full, const char *delim,
                         bool omit_empty_strings,
                         std::vector<std::string> *out);
bool ConvertStringToInteger(const std::string &str, int32 *out);
bool ConvertStringToReal(const std::string &str, float *out);
bool SplitStringToIntegers(const std::string &full, const char *delim,
                           bool omit_empty_strings, std::vector<int32> *out);

}  // namespace kaldi

#endif  // KCNN_KALDI_LITE_KALDI_IO_H_
