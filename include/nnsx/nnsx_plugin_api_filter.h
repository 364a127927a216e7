/*
 * nnsx tensor_filter framework ABI.  Reference:
 * gst/nnstreamer/include/nnstreamer_plugin_api_filter.h:139-495
 * (GstTensorFilterFramework V0: invoke_NN / get{Input,Output}Dimension /
 * setInputDimension / destroyNotify / reloadModel / handleEvent /
 * checkAvailability / allocateInInvoke; V1: open / close / invoke /
 * getFrameworkInfo / getModelInfo / eventHandler with the seven events).
 * Include <nnsx/nnsx_plugin_api.h>.
 *
 * Tables start with a uint32_t version that selects the layout:
 *   NNSX_FILTER_FRAMEWORK_V1  NNSX_FilterFramework without subplugin_data
 *   NNSX_FILTER_FRAMEWORK_V2  NNSX_FilterFramework with subplugin_data: open()
 *                             receives *private_data preset to it (the C++
 *                             base of <nnsx/nnsx_cppplugin_api_filter.hh>)
 *   NNSX_FILTER_FRAMEWORK_V0  NNSX_FilterFrameworkV0 (the legacy table)
 */
#ifndef NNSX_PLUGIN_API_FILTER_H
#define NNSX_PLUGIN_API_FILTER_H

#include <nnsx/nnstreamer_custom.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NNSX_FILTER_FRAMEWORK_V0 0x4e4e5830u /* 'NNX0' */
#define NNSX_FILTER_FRAMEWORK_V1 0x4e4e5831u /* 'NNX1' */
#define NNSX_FILTER_FRAMEWORK_V2 0x4e4e5832u /* 'NNX2' */

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

/* eventHandler events (reference event_ops, nnstreamer_plugin_api_filter.h:199-208).
 * `data` of each event: */
typedef enum {
  NNSX_EVENT_RELOAD_MODEL = 0,          /* const NNSX_FilterProperties * of the new model */
  NNSX_EVENT_CUSTOM = 1,                /* const char * "name=arg" (nnsx: custom downstream events) */
  NNSX_EVENT_CUSTOM_PROP = 2,           /* const NNSX_FilterEventData *: custom_properties */
  NNSX_EVENT_SET_INPUT_PROP = 3,        /* const NNSX_FilterEventData *: info (new input tensors info) */
  NNSX_EVENT_SET_OUTPUT_PROP = 4,       /* const NNSX_FilterEventData *: info (new output tensors info) */
  NNSX_EVENT_SET_ACCELERATOR = 5,       /* const NNSX_FilterEventData *: accelerators ("gpu,cpu"...) */
  NNSX_EVENT_CHECK_HW_AVAILABILITY = 6, /* const NNSX_FilterEventData *: hw ("cpu"/"gpu"), custom;
                                           private_data may be NULL; return 0 = available */
  NNSX_EVENT_DESTROY_NOTIFY = 7,        /* const NNSX_FilterEventData *: data (an allocate-in-invoke
                                           output to free; used when destroyNotify is NULL) */
} NNSX_FilterEvent;

typedef struct {
  const char *custom_properties; /* CUSTOM_PROP */
  const NNSX_TensorsInfo *info;  /* SET_INPUT_PROP / SET_OUTPUT_PROP */
  const char *accelerators;      /* SET_ACCELERATOR: the new accelerator list the framework supports */
  const char *hw;                /* CHECK_HW_AVAILABILITY */
  const char *custom;            /* CHECK_HW_AVAILABILITY: custom option */
  void *data;                    /* DESTROY_NOTIFY */
} NNSX_FilterEventData;

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
  /* V2 only: handed to open() as the initial *private_data */
  void *subplugin_data;
};

/* The legacy V0 table (reference nnstreamer_plugin_api_filter.h:139-262 V0
 * members).  version = NNSX_FILTER_FRAMEWORK_V0; register it with the same
 * entry points (host->register_filter / nnstreamer_filter_probe, cast to
 * const NNSX_FilterFramework *): the runtime dispatches on the version. */
typedef struct _NNSX_FilterFrameworkV0 NNSX_FilterFrameworkV0;
struct _NNSX_FilterFrameworkV0 {
  uint32_t version; /* NNSX_FILTER_FRAMEWORK_V0 */
  const char *name;
  int allow_in_place;
  int allocate_in_invoke;
  int run_without_model;
  int verify_model_path;
  int (*open)(const NNSX_FilterProperties *prop, void **private_data);
  void (*close)(const NNSX_FilterProperties *prop, void **private_data);
  /* host memories (V0 frameworks run on the CPU) */
  int (*invoke_NN)(const NNSX_FilterProperties *prop, void **private_data, const NNSX_TensorMemory *input,
                   NNSX_TensorMemory *output);
  int (*getInputDimension)(const NNSX_FilterProperties *prop, void **private_data, NNSX_TensorsInfo *info);
  int (*getOutputDimension)(const NNSX_FilterProperties *prop, void **private_data, NNSX_TensorsInfo *info);
  int (*setInputDimension)(const NNSX_FilterProperties *prop, void **private_data, const NNSX_TensorsInfo *in_info,
                           NNSX_TensorsInfo *out_info);
  void (*destroyNotify)(void **private_data, void *data);
  int (*reloadModel)(const NNSX_FilterProperties *prop, void **private_data);
  int (*handleEvent)(int event, void **private_data, const void *data); /* NNSX_FilterEvent values */
  int (*checkAvailability)(const char *hw);                            /* 0 = available */
  int (*allocateInInvoke)(void **private_data);                        /* 0 = yes */
};

/* framework=cpp objects (reference ext/nnstreamer/tensor_filter/tensor_filter_cpp.hh):
 * a registered object, found by `model=<name>` (or `model=lib.so,<name>`),
 * reached through these thunks -- <nnsx/tensor_filter_cpp.hh> generates them
 * for a C++ class.  Host memories; invoke's outputs are allocated by the
 * runtime when isAllocatedBeforeInvoke() != 0, else by the object with malloc()
 * (freed by the runtime with free()). */
typedef struct {
  int (*getInputDim)(void *obj, NNSX_TensorsInfo *info);
  int (*getOutputDim)(void *obj, NNSX_TensorsInfo *info);
  int (*setInputDim)(void *obj, const NNSX_TensorsInfo *in, NNSX_TensorsInfo *out);
  int (*isAllocatedBeforeInvoke)(void *obj);
  int (*invoke)(void *obj, const NNSX_TensorMemory *in, NNSX_TensorMemory *out);
} NNSX_CppFilterOps;

#ifdef __cplusplus
}
#endif

#endif /* NNSX_PLUGIN_API_FILTER_H */
