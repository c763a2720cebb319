// euler_amd engine — common layer: Status, logging, string utils, bytes IO.
// Reference counterparts: euler/common/{status.h, error_code.h, logging.h,
// str_util.h, bytes_io.h}.  Written fresh; the
// on-disk byte layout (u32-length-prefixed strings and vectors, little endian)
// is kept so reference-format graph files load unchanged.
#pragma once

#include <stdint.h>
#include <string.h>

#include <atomic>
#include <cstdlib>
#include <functional>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

namespace euler {

// ---------------------------------------------------------------- Status
enum class Code : int {
  OK = 0, CANCELLED = 1, UNKNOWN = 2, INVALID_ARGUMENT = 3, DEADLINE_EXCEEDED = 4, NOT_FOUND = 5,
  ALREADY_EXISTS = 6, PERMISSION_DENIED = 7, RESOURCE_EXHAUSTED = 8, FAILED_PRECONDITION = 9, ABORTED = 10,
  OUT_OF_RANGE = 11, UNIMPLEMENTED = 12, INTERNAL = 13, UNAVAILABLE = 14, DATA_LOSS = 15, UNAUTHENTICATED = 16,
  PROTO_ERROR = 17, RPC_ERROR = 18
};

class Status {
 public:
  Status() = default;
  Status(Code c, std::string msg) : code_(c), msg_(std::move(msg)) {}
  static Status OK() { return Status(); }
  bool ok() const { return code_ == Code::OK; }
  Code code() const { return code_; }
  const std::string& message() const { return msg_; }
  std::string ToString() const;
  static Status Internal(const std::string& m) { return Status(Code::INTERNAL, m); }
  static Status NotFound(const std::string& m) { return Status(Code::NOT_FOUND, m); }
  static Status InvalidArgument(const std::string& m) { return Status(Code::INVALID_ARGUMENT, m); }
  static Status Unavailable(const std::string& m) { return Status(Code::UNAVAILABLE, m); }
  static Status Unimplemented(const std::string& m) { return Status(Code::UNIMPLEMENTED, m); }
  static Status RpcError(const std::string& m) { return Status(Code::RPC_ERROR, m); }
  static Status DataLoss(const std::string& m) { return Status(Code::DATA_LOSS, m); }

 private:
  Code code_ = Code::OK;
  std::string msg_;
};

#define EULER_RETURN_IF_ERROR(expr)          \
  do {                                       \
    ::euler::Status _st = (expr);            \
    if (!_st.ok()) return _st;               \
  } while (0)

// Engine errors surface to Python as exceptions (never exit(), unlike the
// reference parser's yyerror -> exit(1), gremlin.y:272-276).
class EulerError : public std::runtime_error {
 public:
  explicit EulerError(const std::string& m) : std::runtime_error(m) {}
};

// ---------------------------------------------------------------- logging
enum LogSeverity { kDebug = -1, kInfo = 0, kWarning = 1, kError = 2, kFatal = 3 };
int MinLogLevel();  // from EULER_LOG_LEVEL (default: warning)

class LogMessage {
 public:
  LogMessage(const char* file, int line, int sev) : file_(file), line_(line), sev_(sev) {}
  ~LogMessage() noexcept(false);
  std::ostringstream& stream() { return os_; }

 private:
  const char* file_;
  int line_;
  int sev_;
  std::ostringstream os_;
};

#define EULER_LOG(sev)                                             \
  if (::euler::k##sev >= ::euler::MinLogLevel() || ::euler::k##sev == ::euler::kFatal) \
  ::euler::LogMessage(__FILE__, __LINE__, ::euler::k##sev).stream()

#define EULER_CHECK(cond) \
  if (!(cond)) ::euler::LogMessage(__FILE__, __LINE__, ::euler::kFatal).stream() << "Check failed: " #cond " "

#define EULER_THROW(msg)                          \
  do {                                            \
    std::ostringstream _os;                       \
    _os << msg;                                   \
    throw ::euler::EulerError(_os.str());         \
  } while (0)

// ---------------------------------------------------------------- strings
std::vector<std::string> Split(const std::string& s, const std::string& delims, bool skip_empty = true);
std::string Join(const std::vector<std::string>& v, const std::string& sep);
std::string Trim(const std::string& s);
bool StartsWith(const std::string& s, const std::string& p);
bool EndsWith(const std::string& s, const std::string& p);
std::string JoinPath(const std::string& a, const std::string& b);
bool ParseInt64(const std::string& s, int64_t* v);
bool ParseDouble(const std::string& s, double* v);

// ---------------------------------------------------------------- bytes IO
// Little-endian readers/writers for the reference's serialized layout
// (reference euler/common/bytes_io.h: vectors are u32 count + raw elements,
// strings are u32 length + bytes).
class BytesReader {
 public:
  BytesReader(const char* p, size_t n) : p_(p), n_(n) {}
  template <typename T>
  bool Read(T* v) {
    if (pos_ + sizeof(T) > n_) return false;
    memcpy(v, p_ + pos_, sizeof(T));
    pos_ += sizeof(T);
    return true;
  }
  template <typename T>
  bool Read(std::vector<T>* v) {
    uint32_t k = 0;
    if (!Read(&k)) return false;
    if (pos_ + static_cast<size_t>(k) * sizeof(T) > n_) return false;
    v->resize(k);
    if (k) memcpy(v->data(), p_ + pos_, k * sizeof(T));
    pos_ += static_cast<size_t>(k) * sizeof(T);
    return true;
  }
  bool Read(std::string* s) {
    uint32_t k = 0;
    if (!Read(&k)) return false;
    if (pos_ + k > n_) return false;
    s->assign(p_ + pos_, k);
    pos_ += k;
    return true;
  }
  size_t pos() const { return pos_; }
  size_t remaining() const { return n_ - pos_; }
  const char* cur() const { return p_ + pos_; }
  void skip(size_t k) { pos_ += k; }

 private:
  const char* p_;
  size_t n_;
  size_t pos_ = 0;
};

class BytesWriter {
 public:
  BytesWriter() = default;
  // write into caller memory of `cap` bytes instead of the owned string (size() counts
  // every byte offered; overflowed() when that exceeds cap and the tail was dropped)
  BytesWriter(char* ext, size_t cap) : ext_(ext), cap_(cap) {}
  template <typename T>
  void Write(const T& v) {
    WriteRaw(&v, sizeof(T));
  }
  template <typename T>
  void Write(const std::vector<T>& v) {
    Write<uint32_t>(static_cast<uint32_t>(v.size()));
    if (!v.empty()) WriteRaw(v.data(), v.size() * sizeof(T));
  }
  void Write(const std::string& s) {
    Write<uint32_t>(static_cast<uint32_t>(s.size()));
    WriteRaw(s.data(), s.size());
  }
  void WriteRaw(const void* p, size_t n) {
    if (!ext_) {
      buf_.append(static_cast<const char*>(p), n);
      return;
    }
    if (len_ + n <= cap_) memcpy(ext_ + len_, p, n);
    else overflow_ = true;
    len_ += n;
  }
  std::string& str() { return buf_; }
  size_t size() const { return ext_ ? len_ : buf_.size(); }
  bool overflowed() const { return overflow_; }

 private:
  std::string buf_;
  char* ext_ = nullptr;
  size_t cap_ = 0, len_ = 0;
  bool overflow_ = false;
};

// ---------------------------------------------------------------- hash
// MurmurHash3 (public-domain algorithm), bit-compatible with the reference's
// euler/common/hash.{h,cc}: hash64 = first half of x64_128.
uint32_t Hash32(const void* data, int len, uint32_t seed = 0);
void Hash128(const void* data, int len, uint64_t* h1, uint64_t* h2, uint32_t seed = 0);
inline uint64_t Hash64(const void* data, int len, uint32_t seed = 0) {
  uint64_t a, b;
  Hash128(data, len, &a, &b, seed);
  return a;
}
// Edge id hash used by edge attribute indexes (reference data_types.h:48-56).
uint64_t EdgeIdHash(uint64_t src, uint64_t dst, int32_t type);

// ---------------------------------------------------------------- time
uint64_t NowMicros();

}  // namespace euler
