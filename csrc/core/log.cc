#include "core/log.h"

#include <execinfo.h>

#include <cstdio>
#include <cstdlib>
#include <fnmatch.h>
#include <mutex>
#include <vector>

namespace nnsx {
namespace log {

namespace {
struct Rule {
  std::string pattern;
  int level;
};
struct State {
  std::mutex mu;
  std::vector<Rule> rules;
  int default_level = ERROR;
  std::string last_error;
  bool init = false;
};
State& st() {
  static State* s = new State();
  return *s;
}
void parse_spec(State& s, const std::string& spec) {
  s.rules.clear();
  for (auto& item : split(spec, ',')) {
    std::string t = strip(item);
    if (t.empty()) continue;
    auto kv = split(t, ':');
    if (kv.size() == 1) {
      s.default_level = static_cast<int>(to_int(kv[0], ERROR));
    } else {
      int lvl = static_cast<int>(to_int(kv[1], ERROR));
      if (strip(kv[0]) == "*")
        s.default_level = lvl;
      else
        s.rules.push_back({strip(kv[0]), lvl});
    }
  }
}
void ensure_init(State& s) {
  if (s.init) return;
  s.init = true;
  const char* e = std::getenv("NNSX_DEBUG");
  if (!e) e = std::getenv("GST_DEBUG");
  if (e) parse_spec(s, e);
}
}  // namespace

bool enabled(Level lvl, const std::string& category) {
  auto& s = st();
  std::lock_guard<std::mutex> lk(s.mu);
  ensure_init(s);
  int thr = s.default_level;
  for (const auto& r : s.rules)
    if (fnmatch(r.pattern.c_str(), category.c_str(), 0) == 0) thr = r.level;
  return static_cast<int>(lvl) <= thr;
}

void write(Level lvl, const std::string& category, const std::string& msg) {
  static const char* names[] = {"NONE", "ERROR", "WARN", "INFO", "DEBUG", "TRACE"};
  double t = static_cast<double>(now_ns()) / 1e9;
  std::fprintf(stderr, "%.6f %s nnsx %s: %s\n", t, names[lvl], category.c_str(), msg.c_str());
}

void set_threshold(const std::string& spec) {
  auto& s = st();
  std::lock_guard<std::mutex> lk(s.mu);
  s.init = true;
  parse_spec(s, spec);
}

void set_last_error(const std::string& msg) {
  auto& s = st();
  std::lock_guard<std::mutex> lk(s.mu);
  s.last_error = msg.size() > 4096 ? msg.substr(0, 4096) : msg;
}

std::string last_error() {
  auto& s = st();
  std::lock_guard<std::mutex> lk(s.mu);
  return s.last_error;
}

std::string backtrace_string() {
  void* frames[32];
  int n = ::backtrace(frames, 32);
  char** syms = ::backtrace_symbols(frames, n);
  std::string r;
  for (int i = 0; i < n; ++i) {
    r += syms ? syms[i] : "?";
    r += '\n';
  }
  std::free(syms);
  return r;
}

}  // namespace log
}  // namespace nnsx
