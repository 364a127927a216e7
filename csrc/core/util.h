// Small string / parsing helpers shared by the runtime (GLib replacements).
#pragma once

#include <cstdint>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

namespace nnsx {

std::string strip(const std::string& s);
std::string lower(const std::string& s);
std::vector<std::string> split(const std::string& s, char sep, int max_parts = -1);
std::vector<std::string> split_any(const std::string& s, const std::string& seps);
bool starts_with(const std::string& s, const std::string& p);
bool ends_with(const std::string& s, const std::string& p);
std::string join(const std::vector<std::string>& v, const std::string& sep);
std::string replace_all(std::string s, const std::string& from, const std::string& to);

// Lenient numeric parses (g_ascii_strto* semantics: leading spaces ok, garbage -> 0).
int64_t to_int(const std::string& s, int64_t def = 0);
uint64_t to_uint(const std::string& s, uint64_t def = 0);
double to_double(const std::string& s, double def = 0.0);
bool to_bool(const std::string& s, bool def = false);  // true/false/yes/no/1/0/on/off
bool parse_fraction(const std::string& s, int* n, int* d);

template <typename... Args>
std::string strfmt(Args&&... args) {
  std::ostringstream os;
  (os << ... << args);
  return os.str();
}

class Error : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};
// an operation gave up waiting (single-shot invoke timeout; Python: TimeoutError)
class TimeoutError : public Error {
 public:
  using Error::Error;
};

// Monotonic clock in nanoseconds.
int64_t now_ns();
// Wall clock (epoch) in nanoseconds.
int64_t epoch_ns();

constexpr int64_t kClockTimeNone = -1;  // GST_CLOCK_TIME_NONE
constexpr int64_t kSecond = 1000000000LL;

}  // namespace nnsx
