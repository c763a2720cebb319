#include "common/common.h"

#include <sys/time.h>
#include <time.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <iostream>
#include <mutex>

namespace euler {

std::string Status::ToString() const {
  if (ok()) return "OK";
  return "code " + std::to_string(static_cast<int>(code_)) + ": " + msg_;
}

int MinLogLevel() {
  static int lvl = [] {
    const char* e = getenv("EULER_LOG_LEVEL");
    if (!e) return static_cast<int>(kWarning);
    std::string s(e);
    if (s == "debug" || s == "-1") return static_cast<int>(kDebug);
    if (s == "info" || s == "0") return static_cast<int>(kInfo);
    if (s == "warning" || s == "1") return static_cast<int>(kWarning);
    if (s == "error" || s == "2") return static_cast<int>(kError);
    if (s == "fatal" || s == "3") return static_cast<int>(kFatal);
    return static_cast<int>(kWarning);
  }();
  return lvl;
}

LogMessage::~LogMessage() noexcept(false) {
  static const char kSev[] = {'D', 'I', 'W', 'E', 'F'};
  struct timeval tv;
  gettimeofday(&tv, nullptr);
  struct tm tmv;
  localtime_r(&tv.tv_sec, &tmv);
  char ts[64];
  snprintf(ts, sizeof(ts), "%04d-%02d-%02d %02d:%02d:%02d.%06ld", tmv.tm_year + 1900, tmv.tm_mon + 1, tmv.tm_mday,
           tmv.tm_hour, tmv.tm_min, tmv.tm_sec, static_cast<long>(tv.tv_usec));
  const char* base = strrchr(file_, '/');
  base = base ? base + 1 : file_;
  {
    static std::mutex mu;
    std::lock_guard<std::mutex> l(mu);
    std::cerr << ts << ' ' << kSev[sev_ + 1] << ' ' << base << ':' << line_ << "] " << os_.str() << std::endl;
  }
  // FATAL raises (propagates to Python) instead of aborting the whole process.
  if (sev_ == kFatal) throw EulerError(os_.str());
}

std::vector<std::string> Split(const std::string& s, const std::string& delims, bool skip_empty) {
  std::vector<std::string> out;
  std::string cur;
  for (char c : s) {
    if (delims.find(c) != std::string::npos) {
      if (!cur.empty() || !skip_empty) out.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(c);
    }
  }
  if (!cur.empty() || !skip_empty) out.push_back(cur);
  return out;
}

std::string Join(const std::vector<std::string>& v, const std::string& sep) {
  std::string out;
  for (size_t i = 0; i < v.size(); ++i) {
    if (i) out += sep;
    out += v[i];
  }
  return out;
}

std::string Trim(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && isspace(static_cast<unsigned char>(s[a]))) ++a;
  while (b > a && isspace(static_cast<unsigned char>(s[b - 1]))) --b;
  return s.substr(a, b - a);
}

bool StartsWith(const std::string& s, const std::string& p) { return s.compare(0, p.size(), p) == 0; }
bool EndsWith(const std::string& s, const std::string& p) {
  return s.size() >= p.size() && s.compare(s.size() - p.size(), p.size(), p) == 0;
}

std::string JoinPath(const std::string& a, const std::string& b) {
  if (a.empty()) return b;
  if (a.back() == '/') return a + b;
  return a + "/" + b;
}

bool ParseInt64(const std::string& s, int64_t* v) {
  if (s.empty()) return false;
  char* end = nullptr;
  long long x = strtoll(s.c_str(), &end, 10);
  if (end == s.c_str() || *end != '\0') return false;
  *v = x;
  return true;
}

bool ParseDouble(const std::string& s, double* v) {
  if (s.empty()) return false;
  char* end = nullptr;
  double x = strtod(s.c_str(), &end);
  if (end == s.c_str() || *end != '\0') return false;
  *v = x;
  return true;
}

// ---------------------------------------------------------------- MurmurHash3
namespace {
inline uint32_t rotl32(uint32_t x, int8_t r) { return (x << r) | (x >> (32 - r)); }
inline uint64_t rotl64(uint64_t x, int8_t r) { return (x << r) | (x >> (64 - r)); }
inline uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85ebca6b;
  h ^= h >> 13;
  h *= 0xc2b2ae35;
  h ^= h >> 16;
  return h;
}
inline uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}
}  // namespace

uint32_t Hash32(const void* key, int len, uint32_t seed) {
  const uint8_t* data = static_cast<const uint8_t*>(key);
  const int nblocks = len / 4;
  uint32_t h1 = seed;
  const uint32_t c1 = 0xcc9e2d51, c2 = 0x1b873593;
  for (int i = 0; i < nblocks; ++i) {
    uint32_t k1;
    memcpy(&k1, data + i * 4, 4);
    k1 *= c1;
    k1 = rotl32(k1, 15);
    k1 *= c2;
    h1 ^= k1;
    h1 = rotl32(h1, 13);
    h1 = h1 * 5 + 0xe6546b64;
  }
  const uint8_t* tail = data + nblocks * 4;
  uint32_t k1 = 0;
  switch (len & 3) {
    case 3: k1 ^= tail[2] << 16; [[fallthrough]];
    case 2: k1 ^= tail[1] << 8; [[fallthrough]];
    case 1:
      k1 ^= tail[0];
      k1 *= c1;
      k1 = rotl32(k1, 15);
      k1 *= c2;
      h1 ^= k1;
  }
  h1 ^= static_cast<uint32_t>(len);
  return fmix32(h1);
}

void Hash128(const void* key, int len, uint64_t* out1, uint64_t* out2, uint32_t seed) {
  const uint8_t* data = static_cast<const uint8_t*>(key);
  const int nblocks = len / 16;
  uint64_t h1 = seed, h2 = seed;
  const uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
  for (int i = 0; i < nblocks; ++i) {
    uint64_t k1, k2;
    memcpy(&k1, data + i * 16, 8);
    memcpy(&k2, data + i * 16 + 8, 8);
    k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
    h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
    k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
    h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
  }
  const uint8_t* tail = data + nblocks * 16;
  uint64_t k1 = 0, k2 = 0;
  switch (len & 15) {
    case 15: k2 ^= static_cast<uint64_t>(tail[14]) << 48; [[fallthrough]];
    case 14: k2 ^= static_cast<uint64_t>(tail[13]) << 40; [[fallthrough]];
    case 13: k2 ^= static_cast<uint64_t>(tail[12]) << 32; [[fallthrough]];
    case 12: k2 ^= static_cast<uint64_t>(tail[11]) << 24; [[fallthrough]];
    case 11: k2 ^= static_cast<uint64_t>(tail[10]) << 16; [[fallthrough]];
    case 10: k2 ^= static_cast<uint64_t>(tail[9]) << 8; [[fallthrough]];
    case 9:
      k2 ^= static_cast<uint64_t>(tail[8]);
      k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
      [[fallthrough]];
    case 8: k1 ^= static_cast<uint64_t>(tail[7]) << 56; [[fallthrough]];
    case 7: k1 ^= static_cast<uint64_t>(tail[6]) << 48; [[fallthrough]];
    case 6: k1 ^= static_cast<uint64_t>(tail[5]) << 40; [[fallthrough]];
    case 5: k1 ^= static_cast<uint64_t>(tail[4]) << 32; [[fallthrough]];
    case 4: k1 ^= static_cast<uint64_t>(tail[3]) << 24; [[fallthrough]];
    case 3: k1 ^= static_cast<uint64_t>(tail[2]) << 16; [[fallthrough]];
    case 2: k1 ^= static_cast<uint64_t>(tail[1]) << 8; [[fallthrough]];
    case 1:
      k1 ^= static_cast<uint64_t>(tail[0]);
      k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
  }
  h1 ^= static_cast<uint64_t>(len);
  h2 ^= static_cast<uint64_t>(len);
  h1 += h2;
  h2 += h1;
  h1 = fmix64(h1);
  h2 = fmix64(h2);
  h1 += h2;
  h2 += h1;
  *out1 = h1;
  *out2 = h2;
}

uint64_t EdgeIdHash(uint64_t src, uint64_t dst, int32_t type) {
  char tmp[20];
  memcpy(tmp, &src, 8);
  memcpy(tmp + 8, &dst, 8);
  memcpy(tmp + 16, &type, 4);
  return Hash64(tmp, 20);
}

uint64_t NowMicros() {
  return std::chrono::duration_cast<std::chrono::microseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

}  // namespace euler
