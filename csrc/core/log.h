// Logging (ml_log{i,w,e,d} equivalent) with a GST_DEBUG-style env var and the
// global last-error buffer of gst/nnstreamer/nnstreamer_log.c:71-128.
//   NNSX_DEBUG="*:2,tensor_filter*:5"   levels: 0 none 1 error 2 warn 3 info 4 debug 5 trace
#pragma once

#include <string>

#include "core/util.h"

namespace nnsx {
namespace log {

enum Level { NONE = 0, ERROR = 1, WARN = 2, INFO = 3, DEBUG = 4, TRACE = 5 };

bool enabled(Level lvl, const std::string& category);
void write(Level lvl, const std::string& category, const std::string& msg);
void set_threshold(const std::string& spec);  // same syntax as NNSX_DEBUG
// last error (nnstreamer's _nnstreamer_error())
void set_last_error(const std::string& msg);
std::string last_error();
std::string backtrace_string();

}  // namespace log
}  // namespace nnsx

#define NNSX_LOG_(lvl, cat, ...)                                                     \
  do {                                                                               \
    if (::nnsx::log::enabled(lvl, cat)) ::nnsx::log::write(lvl, cat, ::nnsx::strfmt(__VA_ARGS__)); \
  } while (0)
#define NNSX_LOGE(cat, ...)                                         \
  do {                                                              \
    std::string _m = ::nnsx::strfmt(__VA_ARGS__);                   \
    ::nnsx::log::set_last_error(_m);                                \
    if (::nnsx::log::enabled(::nnsx::log::ERROR, cat)) ::nnsx::log::write(::nnsx::log::ERROR, cat, _m); \
  } while (0)
#define NNSX_LOGW(cat, ...) NNSX_LOG_(::nnsx::log::WARN, cat, __VA_ARGS__)
#define NNSX_LOGI(cat, ...) NNSX_LOG_(::nnsx::log::INFO, cat, __VA_ARGS__)
#define NNSX_LOGD(cat, ...) NNSX_LOG_(::nnsx::log::DEBUG, cat, __VA_ARGS__)
