// kaldi-lite/kaldi-io.cc
#include "kaldi-io.h"

#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include <iomanip>
#include <limits>

namespace kaldi {

void WriteToken(std::ostream &os, bool binary, const std::string &token) {
  (void)binary;
  if (token.empty() || token.find(' ') != std::string::npos)
    KALDI_ERR << "invalid token '" << token << "'";
  os << token << " ";
  if (os.fail()) KALDI_ERR << "write failure in WriteToken";
}

void ReadToken(std::istream &is, bool binary, std::string *token) {
  if (!binary) is >> std::ws;
  is >> *token;
  if (is.fail()) KALDI_ERR << "ReadToken: failed to read token";
  if (!isspace(is.peek()))
    KALDI_ERR << "ReadToken: expected space after token, saw "
              << (char)is.peek();
  is.get();
}

void ExpectToken(std::istream &is, bool binary, const std::string &token) {
  std::string got;
  ReadToken(is, binary, &got);
  if (got != token)
    KALDI_ERR << "Expected token \"" << token << "\", got \"" << got << "\"";
}

int PeekToken(std::istream &is, bool binary) {
  if (!binary) is >> std::ws;
  bool read_bracket;
  if ((read_bracket = (static_cast<char>(is.peek()) == '<'))) is.get();
  int ans = is.peek();
  if (read_bracket) is.unget();
  return ans;
}

template <typename T>
static void write_raw(std::ostream &os, T t) {
  os.put((char)sizeof(T));
  os.write(reinterpret_cast<const char *>(&t), sizeof(T));
}
template <typename T>
static void read_raw(std::istream &is, T *t) {
  const int len = is.get();
  if (len != (int)sizeof(T))
    KALDI_ERR << "ReadBasicType: expected size byte " << sizeof(T) << ", got "
              << len;
  is.read(reinterpret_cast<char *>(t), sizeof(T));
  if (is.fail()) KALDI_ERR << "ReadBasicType: read failure";
}

void WriteBasicType(std::ostream &os, bool binary, int32 t) {
  if (binary) write_raw(os, t);
  else os << t << " ";
}
void WriteBasicType(std::ostream &os, bool binary, float t) {
  if (binary) write_raw(os, t);
  else os << std::setprecision(std::numeric_limits<float>::max_digits10) << t << " ";
}
void WriteBasicType(std::ostream &os, bool binary, bool t) {
  os << (t ? "T" : "F");
  if (!binary) os << " ";
}
void ReadBasicType(std::istream &is, bool binary, int32 *t) {
  if (binary) read_raw(is, t);
  else { is >> *t; if (is.fail()) KALDI_ERR << "ReadBasicType<int32> failed"; }
}
void ReadBasicType(std::istream &is, bool binary, float *t) {
  if (binary) {
    read_raw(is, t);
  } else {
    std::string s;
    is >> s;
    if (is.fail() || !ConvertStringToReal(s, t))
      KALDI_ERR << "ReadBasicType<float> failed on '" << s << "'";
  }
}
void WriteBasicType(std::ostream &os, bool binary, double t) {
  if (binary) write_raw(os, t);
  else os << std::setprecision(std::numeric_limits<double>::max_digits10) << t << " ";
}
void ReadBasicType(std::istream &is, bool binary, double *t) {
  if (binary) {
    read_raw(is, t);
  } else {
    std::string s;
    is >> s;
    char *end = nullptr;
    *t = strtod(s.c_str(), &end);
    if (is.fail() || s.empty() || *end != '\0')
      KALDI_ERR << "ReadBasicType<double> failed on '" << s << "'";
  }
}
void WriteIntegerVector(std::ostream &os, bool binary, const std::vector<int32> &v) {
  if (binary) {
    const char sz = sizeof(int32);
    os.write(&sz, 1);
    const int32 n = (int32)v.size();
    os.write(reinterpret_cast<const char *>(&n), sizeof(n));
    if (n) os.write(reinterpret_cast<const char *>(v.data()), sizeof(int32) * n);
  } else {
    os << "[ ";
    for (int32 x : v) os << x << " ";
    os << "]\n";
  }
  if (os.fail()) KALDI_ERR << "WriteIntegerVector: write failure";
}
void ReadIntegerVector(std::istream &is, bool binary, std::vector<int32> *v) {
  v->clear();
  if (binary) {
    char sz = 0;
    is.read(&sz, 1);
    if (sz != (char)sizeof(int32))
      KALDI_ERR << "ReadIntegerVector: expected size byte 4, got " << (int)sz;
    int32 n = 0;
    is.read(reinterpret_cast<char *>(&n), sizeof(n));
    if (is.fail() || n < 0) KALDI_ERR << "ReadIntegerVector: bad size";
    v->resize(n);
    if (n) is.read(reinterpret_cast<char *>(v->data()), sizeof(int32) * n);
    if (is.fail()) KALDI_ERR << "ReadIntegerVector: read failure";
    return;
  }
  std::string tok;
  is >> tok;
  if (tok != "[") KALDI_ERR << "ReadIntegerVector: expected '[', got " << tok;
  while (is >> tok) {
    if (tok == "]") { is >> std::ws; return; }
    int32 x;
    if (!ConvertStringToInteger(tok, &x)) KALDI_ERR << "ReadIntegerVector: bad value " << tok;
    v->push_back(x);
  }
  KALDI_ERR << "ReadIntegerVector: unterminated vector";
}
void ReadBasicType(std::istream &is, bool binary, bool *t) {
  if (!binary) is >> std::ws;
  const char c = is.peek();
  if (c == 'T') *t = true;
  else if (c == 'F') *t = false;
  else KALDI_ERR << "ReadBasicType<bool>: expected T or F, got " << c;
  is.get();
  if (!binary) is >> std::ws;
}

void InitKaldiOutputStream(std::ostream &os, bool binary) {
  if (binary) { os.put('\0'); os.put('B'); }
  os.precision(7);
}
bool InitKaldiInputStream(std::istream &is, bool *binary) {
  if (is.peek() == '\0') {
    is.get();
    if (is.peek() != 'B') return false;
    is.get();
    *binary = true;
    return true;
  }
  *binary = false;
  return true;
}

void SplitStringToVector(const std::string &full, const char *delim,
                         bool omit_empty_strings,
                         std::vector<std::string> *out) {
  out->clear();
  size_t start = 0, found = 0, end = full.size();
  while (found != std::string::npos) {
    found = full.find_first_of(delim, start);
    if (!omit_empty_strings || (found != start && start != end))
      out->push_back(full.substr(start, found - start));
    start = found + 1;
  }
}

bool ConvertStringToInteger(const std::string &str, int32 *out) {
  const char *p = str.c_str();
  char *end = nullptr;
  errno = 0;
  long v = strtol(p, &end, 10);
  while (end && isspace(*end)) end++;
  if (end == p || *end != '\0' || errno != 0) return false;
  if (v < std::numeric_limits<int32>::min() || v > std::numeric_limits<int32>::max())
    return false;
  *out = (int32)v;
  return true;
}

bool ConvertStringToReal(const std::string &str, float *out) {
  const char *p = str.c_str();
  char *end = nullptr;
  double v = strtod(p, &end);
  while (end && isspace(*end)) end++;
  if (end == p || *end != '\0') return false;
  *out = (float)v;
  return true;
}

bool SplitStringToIntegers(const std::string &full, const char *delim,
                           bool omit_empty_strings, std::vector<int32> *out) {
  std::vector<std::string> parts;
  SplitStringToVector(full, delim, omit_empty_strings, &parts);
  out->clear();
  for (auto &s : parts) {
    int32 v;
    if (!ConvertStringToInteger(s, &v)) { out->clear(); return false; }
    out->push_back(v);
  }
  return true;
}

}  // namespace kaldi
