/*
 * nnsx tensor_filter framework ABI (V1 style).  Reference:
 * gst/nnstreamer/include/nnstreamer_plugin_api_filter.h:273-495
 * (GstTensorFilterFramework V1: open / close / invoke / getFrameworkInfo /
 * getModelInfo / eventHandler).  Include <nnsx/nnsx_plugin_api.h>.
 */
#ifndef NNSX_PLUGIN_API_FILTER_H
#define NNSX_PLUGIN_API_FILTER_H

#include <nnsx/nnstreamer_custom.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NNSX_FILTER_FRAMEWORK_V1 0x4e4e5831u /* 'NNX1' */

/* where an invoke runs: device -1 = host memories; else the GPU index, and
 * input/output data pointers are device pointers ordered on `stream` (a
 * hipStream_t): enqueue work on it, do not synchronise unless needed */
typedef struct {
  int device;
  void *stream;
} NNSX_InvokeContext;

typedef enum {
  NNSX_GET_IN_OUT_INFO = 0, /* report the model's fixed input and output info */
  NNSX_SET_INPUT_INFO = 1,  /* in_info is given: report the matching out_info */
} NNSX_ModelInfoOps;

typedef enum {
  NNSX_EVENT_RELOAD_MODEL = 0, /* data: const NNSX_FilterProperties * of the new model */
  NNSX_EVENT_CUSTOM = 1,       /* data: const char * "name=arg" */
} NNSX_FilterEvent;

typedef struct {
  const char *name;
  int allocate_in_invoke; /* 1: invoke allocates outputs, destroyNotify frees them */
  int run_without_model;
  int verify_model_path;
  const char *accelerators;     /* e.g. "cpu" or "gpu,cpu" */
  const char *model_extensions; /* e.g. ".pt,.pth" (framework=auto detection) */
} NNSX_FrameworkInfo;

struct _NNSX_FilterFramework {
  uint32_t version; /* NNSX_FILTER_FRAMEWORK_V1 */
  const char *name;
  /* prop->model_files etc.; store per-instance state in *private_data */
  int (*open)(const NNSX_FilterProperties *prop, void **private_data);
  void (*close)(const NNSX_FilterProperties *prop, void **private_data);
  int (*getFrameworkInfo)(const NNSX_FilterFramework *self, const NNSX_FilterProperties *prop, void *private_data,
                          NNSX_FrameworkInfo *info);
  int (*getModelInfo)(const NNSX_FilterFramework *self, const NNSX_FilterProperties *prop, void *private_data,
                      NNSX_ModelInfoOps ops, NNSX_TensorsInfo *in_info, NNSX_TensorsInfo *out_info);
  /* output[i].data: pre-allocated by the runtime (host, or device memory of
   * ctx->device) unless allocate_in_invoke, in which case the framework sets
   * data/size and the runtime calls destroyNotify(private_data, data) once the
   * last reader is done */
  int (*invoke)(const NNSX_FilterFramework *self, const NNSX_FilterProperties *prop, void *private_data,
                const NNSX_TensorMemory *input, NNSX_TensorMemory *output, const NNSX_InvokeContext *ctx);
  void (*destroyNotify)(void *private_data, void *data);
  /* optional; return 0 if handled, -ENOENT (-2) if not supported */
  int (*eventHandler)(const NNSX_FilterFramework *self, const NNSX_FilterProperties *prop, void *private_data,
                      NNSX_FilterEvent event, const void *data);
};

#ifdef __cplusplus
}
#endif

#endif /* NNSX_PLUGIN_API_FILTER_H */
