// Entry shim of the native command-line tools (bin/nnsx-launch, bin/nnsx-check).
//
// The runtime library links PyTorch-ROCm, which ships its own HIP runtime and
// RCCL.  A Python process always loads torch first, so libnnsx's HIP/RCCL
// dependencies resolve to torch's copies; a plain executable linked against
// libnnsx would instead pull the system ROCm copies as well (same SONAME,
// different file) and run two HIP runtimes side by side.  The shim loads the
// torch runtime first, then libnnsx, and calls the tool's entry point.
#include <dlfcn.h>
#include <limits.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <string>

#ifndef NNSX_TOOL_ENTRY
#error "NNSX_TOOL_ENTRY (the tool's entry symbol) must be defined"
#endif
#ifndef NNSX_TORCH_LIB
#error "NNSX_TORCH_LIB (PyTorch's lib directory) must be defined"
#endif
#define NNSX_STR2(x) #x
#define NNSX_STR(x) NNSX_STR2(x)

static std::string exe_dir() {
  char buf[PATH_MAX];
  const ssize_t n = readlink("/proc/self/exe", buf, sizeof(buf) - 1);
  if (n <= 0) return ".";
  buf[n] = 0;
  std::string p(buf);
  return p.substr(0, p.rfind('/'));
}

int main(int argc, char** argv) {
  const std::string torch = NNSX_TORCH_LIB;
  for (const char* lib : {"libamdhip64.so", "librccl.so", "libtorch_hip.so"}) {
    if (!dlopen((torch + "/" + lib).c_str(), RTLD_NOW | RTLD_GLOBAL)) {
      std::fprintf(stderr, "cannot load %s/%s: %s\n", torch.c_str(), lib, dlerror());
      return 2;
    }
  }
  const std::string lib = exe_dir() + "/../nnstreamer_amd/libnnsx.so";
  void* h = dlopen(lib.c_str(), RTLD_NOW | RTLD_GLOBAL);
  if (!h) {
    std::fprintf(stderr, "cannot load %s: %s (build it: python nnstreamer_amd/_build.py)\n", lib.c_str(), dlerror());
    return 2;
  }
  auto entry = reinterpret_cast<int (*)(int, char**)>(dlsym(h, NNSX_STR(NNSX_TOOL_ENTRY)));
  if (!entry) {
    std::fprintf(stderr, "%s: no entry point %s\n", lib.c_str(), NNSX_STR(NNSX_TOOL_ENTRY));
    return 2;
  }
  return entry(argc, argv);
}
