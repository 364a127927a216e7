// nnsx-launch: run a pipeline description, gst-launch-1.0 style, natively
// (reference: GStreamer's gst-launch as used by every tests/*/runTest.sh).
//
//   nnsx-launch [-v] [-m] [-e] [-t SEC] [--dot FILE] [--debug LEVEL] DESCRIPTION...
//
// Exit status: 0 EOS, 1 error message on the bus, 2 parse / state failure,
// 3 timeout, 130 interrupted.  -v prints the negotiated caps of every pad at
// the end, -m every bus message, -e turns SIGINT into an EOS at the sources
// (clean shutdown) instead of stopping at once.
#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "core/log.h"
#include "core/util.h"
#include "runtime/pipeline.h"

using namespace nnsx;

namespace {

volatile std::sig_atomic_t g_interrupted = 0;
void on_sigint(int) { g_interrupted = 1; }

int usage() {
  std::fprintf(stderr,
               "usage: nnsx-launch [-v] [-m] [-e] [-t SEC] [--dot FILE] [--debug LEVEL] PIPELINE-DESCRIPTION\n");
  return 2;
}

}  // namespace

extern "C" __attribute__((visibility("default"))) int nnsx_launch_main(int argc, char** argv) {
  bool verbose = false, messages = false, eos_on_int = false;
  double timeout_s = 0;
  std::string dot_path, debug;
  std::vector<std::string> parts;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "-v" || a == "--verbose") verbose = true;
    else if (a == "-m" || a == "--messages") messages = true;
    else if (a == "-e" || a == "--eos-on-shutdown") eos_on_int = true;
    else if ((a == "-t" || a == "--timeout") && i + 1 < argc) timeout_s = std::atof(argv[++i]);
    else if (a == "--dot" && i + 1 < argc) dot_path = argv[++i];
    else if (a == "--debug" && i + 1 < argc) debug = argv[++i];
    else if (a == "-h" || a == "--help") return usage() - 2;
    else parts.push_back(a);
  }
  if (parts.empty()) return usage();
  if (!debug.empty()) log::set_threshold(debug);
  std::string desc;
  for (auto& p : parts) desc += (desc.empty() ? "" : " ") + p;

  std::unique_ptr<Pipeline> p;
  try {
    p = parse_launch(desc);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "ERROR: pipeline could not be constructed: %s\n", e.what());
    return 2;
  }
  std::signal(SIGINT, on_sigint);
  const int64_t t0 = now_ns();
  std::printf("Setting pipeline to PLAYING ...\n");
  std::fflush(stdout);
  if (!p->set_state(State::PLAYING)) {
    std::fprintf(stderr, "ERROR: pipeline doesn't want to play: %s\n", log::last_error().c_str());
    p->set_state(State::NULL_);
    return 2;
  }
  int rc = 3;
  bool eos_sent = false;
  while (true) {
    if (g_interrupted && !eos_sent) {
      if (!eos_on_int) {
        std::fprintf(stderr, "Interrupt: stopping pipeline ...\n");
        rc = 130;
        break;
      }
      std::fprintf(stderr, "Interrupt: sending EOS ...\n");
      p->send_eos();
      eos_sent = true;
    }
    if (timeout_s > 0 && now_ns() - t0 > static_cast<int64_t>(timeout_s * 1e9)) {
      std::fprintf(stderr, "Timed out after %.1f s\n", timeout_s);
      rc = 3;
      break;
    }
    Message m;
    if (!p->bus().pop(&m, 100000000)) continue;  // 100 ms slices: signals and timeout stay responsive
    if (messages)
      std::printf("Got message from \"%s\": %s %s\n", m.src.c_str(), message_type_name(m.type), m.text.c_str());
    if (m.type == MessageType::ERROR) {
      std::fprintf(stderr, "ERROR: from element %s: %s\n", m.src.c_str(), m.text.c_str());
      rc = 1;
      break;
    }
    if (m.type == MessageType::EOS) {
      std::printf("Got EOS from pipeline. Execution ended after %.9f s\n", (now_ns() - t0) / 1e9);
      rc = 0;
      break;
    }
  }
  if (verbose)
    for (Element* e : p->elements())
      for (auto& pad : e->pads())
        if (pad->has_current_caps())
          std::printf("/%s:%s: caps = %s\n", e->name().c_str(), pad->name().c_str(),
                      pad->current_caps().to_string().c_str());
  if (!dot_path.empty()) {
    std::ofstream f(dot_path);
    f << p->dot();
  }
  std::printf("Setting pipeline to NULL ...\n");
  p->set_state(State::NULL_);
  return rc;
}
