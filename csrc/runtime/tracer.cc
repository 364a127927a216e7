// Built-in tracers.  See tracer.h.
#include "runtime/tracer.h"

#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <sstream>
#include <vector>

#include "core/util.h"
#include "runtime/element.h"

namespace nnsx {
namespace trace {

std::atomic<uint32_t> g_flags{0};

namespace {

struct Stats {
  uint64_t buffers = 0;
  int64_t first_ns = -1, last_ns = -1;
  uint64_t proc_n = 0;
  int64_t proc_sum = 0, proc_min = INT64_MAX, proc_max = 0;
  uint64_t lat_n = 0;
  int64_t lat_sum = 0, lat_max = 0, lat_last = 0;
};

std::mutex g_mu;
std::map<std::string, Stats> g_stats;

// per-thread stack of elements whose chain is running (a queue / source
// thread pushes through a run of elements nested in each other's chain)
struct Frame {
  Element* elem;
  int64_t enter_ns;
  bool pushed;
};
thread_local std::vector<Frame> t_stack;

void record_proc(Element* e, int64_t dt) {
  std::lock_guard<std::mutex> lk(g_mu);
  Stats& s = g_stats[e->name()];
  ++s.proc_n;
  s.proc_sum += dt;
  s.proc_min = std::min(s.proc_min, dt);
  s.proc_max = std::max(s.proc_max, dt);
}

struct EnvInit {
  EnvInit() {
    if (const char* e = std::getenv("NNSX_TRACERS")) enable(e);
  }
} g_env_init;

}  // namespace

void enable(const std::string& spec) {
  uint32_t f = 0;
  for (auto& t : split(spec, ';')) {
    const std::string n = strip(t);
    if (n == "proctime") f |= PROCTIME;
    else if (n == "interlatency") f |= INTERLATENCY;
    else if (n == "framerate") f |= FRAMERATE;
    else if (n == "roctx") f |= ROCTX;
    else if (n == "all") f |= PROCTIME | INTERLATENCY | FRAMERATE;
  }
  g_flags.store(f);
}

void reset() {
  std::lock_guard<std::mutex> lk(g_mu);
  g_stats.clear();
}

void chain_enter(Element* e, int64_t origin_ns) {
  const uint32_t f = flags();
  const int64_t now = now_ns();
  if (f & ROCTX) roctxRangePushA(e->name().c_str());
  if (f & (FRAMERATE | INTERLATENCY)) {
    std::lock_guard<std::mutex> lk(g_mu);
    Stats& s = g_stats[e->name()];
    ++s.buffers;
    if (s.first_ns < 0) s.first_ns = now;
    s.last_ns = now;
    if ((f & INTERLATENCY) && origin_ns >= 0) {
      const int64_t l = now - origin_ns;
      ++s.lat_n;
      s.lat_sum += l;
      s.lat_max = std::max(s.lat_max, l);
      s.lat_last = l;
    }
  }
  t_stack.push_back(Frame{e, now, false});
}

void chain_exit(Element* e) {
  const uint32_t f = flags();
  if (f & ROCTX) roctxRangePop();
  if (t_stack.empty() || t_stack.back().elem != e) return;
  const Frame fr = t_stack.back();
  t_stack.pop_back();
  // an element that pushed nothing (a sink, or one that queued the buffer): its whole chain
  if ((f & PROCTIME) && !fr.pushed) record_proc(e, now_ns() - fr.enter_ns);
}

void src_push(Element* e) {
  if (!(flags() & PROCTIME)) return;
  for (auto it = t_stack.rbegin(); it != t_stack.rend(); ++it)
    if (it->elem == e) {
      if (!it->pushed) {
        it->pushed = true;
        record_proc(e, now_ns() - it->enter_ns);
      }
      return;
    }
}

std::string report_json() {
  std::lock_guard<std::mutex> lk(g_mu);
  std::ostringstream os;
  os << "{\"tracers\": [";
  const uint32_t f = flags();
  bool first = true;
  for (auto& n : {std::make_pair(PROCTIME, "proctime"), std::make_pair(INTERLATENCY, "interlatency"),
                  std::make_pair(FRAMERATE, "framerate"), std::make_pair(ROCTX, "roctx")})
    if (f & n.first) {
      os << (first ? "" : ", ") << "\"" << n.second << "\"";
      first = false;
    }
  os << "], \"elements\": {";
  first = true;
  for (auto& kv : g_stats) {
    const Stats& s = kv.second;
    os << (first ? "" : ", ") << "\"" << kv.first << "\": {\"buffers\": " << s.buffers;
    if (s.buffers > 1 && s.last_ns > s.first_ns)
      os << ", \"fps\": " << (static_cast<double>(s.buffers - 1) * 1e9 / static_cast<double>(s.last_ns - s.first_ns));
    if (s.proc_n)
      os << ", \"proctime_us\": {\"n\": " << s.proc_n << ", \"avg\": " << (s.proc_sum / 1e3 / s.proc_n)
         << ", \"min\": " << s.proc_min / 1e3 << ", \"max\": " << s.proc_max / 1e3 << "}";
    if (s.lat_n)
      os << ", \"interlatency_us\": {\"n\": " << s.lat_n << ", \"avg\": " << (s.lat_sum / 1e3 / s.lat_n)
         << ", \"max\": " << s.lat_max / 1e3 << ", \"last\": " << s.lat_last / 1e3 << "}";
    os << "}";
    first = false;
  }
  os << "}}";
  return os.str();
}

}  // namespace trace
}  // namespace nnsx
