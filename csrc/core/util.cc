#include "core/util.h"

#include <algorithm>
#include <cctype>
#include <chrono>
#include <cstdlib>

namespace nnsx {

std::string strip(const std::string& s) {
  size_t b = 0, e = s.size();
  while (b < e && std::isspace(static_cast<unsigned char>(s[b]))) ++b;
  while (e > b && std::isspace(static_cast<unsigned char>(s[e - 1]))) --e;
  return s.substr(b, e - b);
}

std::string lower(const std::string& s) {
  std::string r = s;
  std::transform(r.begin(), r.end(), r.begin(), [](unsigned char c) { return std::tolower(c); });
  return r;
}

std::vector<std::string> split(const std::string& s, char sep, int max_parts) {
  std::vector<std::string> out;
  size_t start = 0;
  while (true) {
    if (max_parts > 0 && static_cast<int>(out.size()) == max_parts - 1) {
      out.push_back(s.substr(start));
      break;
    }
    size_t p = s.find(sep, start);
    if (p == std::string::npos) {
      out.push_back(s.substr(start));
      break;
    }
    out.push_back(s.substr(start, p - start));
    start = p + 1;
  }
  return out;
}

std::vector<std::string> split_any(const std::string& s, const std::string& seps) {
  std::vector<std::string> out;
  std::string cur;
  for (char c : s) {
    if (seps.find(c) != std::string::npos) {
      out.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(c);
    }
  }
  out.push_back(cur);
  return out;
}

bool starts_with(const std::string& s, const std::string& p) { return s.compare(0, p.size(), p) == 0; }
bool ends_with(const std::string& s, const std::string& p) {
  return s.size() >= p.size() && s.compare(s.size() - p.size(), p.size(), p) == 0;
}

std::string join(const std::vector<std::string>& v, const std::string& sep) {
  std::string r;
  for (size_t i = 0; i < v.size(); ++i) {
    if (i) r += sep;
    r += v[i];
  }
  return r;
}

std::string replace_all(std::string s, const std::string& from, const std::string& to) {
  if (from.empty()) return s;
  size_t p = 0;
  while ((p = s.find(from, p)) != std::string::npos) {
    s.replace(p, from.size(), to);
    p += to.size();
  }
  return s;
}

int64_t to_int(const std::string& s, int64_t def) {
  std::string t = strip(s);
  if (t.empty()) return def;
  char* end = nullptr;
  long long v = std::strtoll(t.c_str(), &end, 0);
  if (end == t.c_str()) return def;
  return v;
}

uint64_t to_uint(const std::string& s, uint64_t def) {
  std::string t = strip(s);
  if (t.empty()) return def;
  char* end = nullptr;
  unsigned long long v = std::strtoull(t.c_str(), &end, 10);
  if (end == t.c_str()) return def;
  return v;
}

double to_double(const std::string& s, double def) {
  std::string t = strip(s);
  if (t.empty()) return def;
  char* end = nullptr;
  double v = std::strtod(t.c_str(), &end);
  if (end == t.c_str()) return def;
  return v;
}

bool to_bool(const std::string& s, bool def) {
  std::string t = lower(strip(s));
  if (t == "true" || t == "yes" || t == "1" || t == "on" || t == "t" || t == "y") return true;
  if (t == "false" || t == "no" || t == "0" || t == "off" || t == "f" || t == "n") return false;
  return def;
}

bool parse_fraction(const std::string& s, int* n, int* d) {
  auto parts = split(strip(s), '/');
  if (parts.empty() || parts.size() > 2) return false;
  std::string a = strip(parts[0]);
  if (a.empty()) return false;
  *n = static_cast<int>(to_int(a));
  *d = parts.size() == 2 ? static_cast<int>(to_int(parts[1], 1)) : 1;
  return true;
}

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int64_t epoch_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::system_clock::now().time_since_epoch())
      .count();
}

}  // namespace nnsx
