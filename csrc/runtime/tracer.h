// Built-in pipeline tracers (the reference has none of its own and points to
// GstShark / gst-instruments: tools/tracing/README.md, tools/profiling/README.md).
//
//   NNSX_TRACERS="proctime;interlatency;framerate;roctx"   (or tracer_enable())
//
// * proctime     per element: time from a buffer entering the element (its
//                chain) to the element's first push downstream (GstShark
//                proctime); sinks: time inside render.
// * interlatency per element: time from the buffer's origin (the first push
//                at a source; copied through copy_metadata_from) to its
//                arrival at the element (GstShark interlatency).
// * framerate    buffers per second through every element (over the run).
// * roctx        one roctx range per element chain call, so a
//                `rocprofv3 --marker-trace --kernel-trace` timeline shows the
//                pipeline stages over the kernels they launch.
//
// Hooks live in Pad::push (one relaxed atomic load when tracing is off).
// tracer_report() returns JSON: {"elements": {name: {...}}, ...}.
// NNSX_DEBUG_DUMP_DOT_DIR=<dir> writes <dir>/<pipeline>.<state>.dot on state
// changes (GST_DEBUG_DUMP_DOT_DIR analogue).
#pragma once

#include <atomic>
#include <cstdint>
#include <string>

namespace nnsx {

class Element;

namespace trace {

enum Flags : uint32_t { PROCTIME = 1, INTERLATENCY = 2, FRAMERATE = 4, ROCTX = 8 };

extern std::atomic<uint32_t> g_flags;
inline uint32_t flags() { return g_flags.load(std::memory_order_relaxed); }

void enable(const std::string& spec);  // "proctime;interlatency" ("" / "none" disables)
void reset();
std::string report_json();

// Pad::push hooks: the buffer enters `sink_elem` (called before its chain)...
void chain_enter(Element* sink_elem, int64_t origin_ns);
// ...and leaves it (chain returned)
void chain_exit(Element* sink_elem);
// `src_elem` pushes a buffer downstream (proctime ends at its first push)
void src_push(Element* src_elem);

}  // namespace trace
}  // namespace nnsx
