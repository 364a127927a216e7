/*
 * nnsx custom-filter C ABI (framework=custom model=libfoo.so).
 *
 * Same shape as NNStreamer's NNStreamer_custom_class
 * (gst/nnstreamer/include/tensor_filter_custom.h:125-136): the shared object
 * exports `NNStreamer_custom`, a table of callbacks.  The tensor-info structs
 * are plain C (no GLib), dimensions innermost-first, type codes equal to the
 * NNStreamer enum order (int32=0 ... float16=10, nnsx bfloat16=12).
 */
#ifndef NNSX_TENSOR_FILTER_CUSTOM_H
#define NNSX_TENSOR_FILTER_CUSTOM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NNSX_RANK_LIMIT 8
#define NNSX_SIZE_LIMIT 16

typedef struct {
  char *name;
  uint32_t type;
  uint32_t dimension[NNSX_RANK_LIMIT];
} NNSX_TensorInfo;

typedef struct {
  uint32_t num_tensors;
  NNSX_TensorInfo info[NNSX_SIZE_LIMIT];
  uint32_t format; /* 0 static, 1 flexible, 2 sparse */
} NNSX_TensorsInfo;

typedef struct {
  void *data;
  size_t size;
} NNSX_TensorMemory;

typedef struct {
  const char *fwname;
  const char **model_files;
  int num_models;
  const char *custom_properties;
  NNSX_TensorsInfo input_meta;
  NNSX_TensorsInfo output_meta;
} NNSX_FilterProperties;

typedef void *(*NNS_custom_init_func)(const NNSX_FilterProperties *prop);
typedef void (*NNS_custom_exit_func)(void *private_data, const NNSX_FilterProperties *prop);
typedef int (*NNS_custom_get_input_dimension)(void *private_data, const NNSX_FilterProperties *prop,
                                              NNSX_TensorsInfo *info);
typedef int (*NNS_custom_get_output_dimension)(void *private_data, const NNSX_FilterProperties *prop,
                                               NNSX_TensorsInfo *info);
typedef int (*NNS_custom_set_input_dimension)(void *private_data, const NNSX_FilterProperties *prop,
                                              const NNSX_TensorsInfo *in_info, NNSX_TensorsInfo *out_info);
typedef int (*NNS_custom_invoke)(void *private_data, const NNSX_FilterProperties *prop,
                                 const NNSX_TensorMemory *input, NNSX_TensorMemory *output);
typedef int (*NNS_custom_allocate_invoke)(void *private_data, const NNSX_FilterProperties *prop,
                                          const NNSX_TensorMemory *input, NNSX_TensorMemory *output);
typedef void (*NNS_custom_destroy_notify)(void *data);

typedef struct {
  NNS_custom_init_func initfunc;
  NNS_custom_exit_func exitfunc;
  NNS_custom_get_input_dimension getInputDim;
  NNS_custom_get_output_dimension getOutputDim;
  NNS_custom_set_input_dimension setInputDim;
  NNS_custom_invoke invoke;
  NNS_custom_allocate_invoke allocate_invoke;
  NNS_custom_destroy_notify destroy_notify;
} NNStreamer_custom_class;

extern NNStreamer_custom_class *NNStreamer_custom;

#ifdef __cplusplus
}
#endif

#endif /* NNSX_TENSOR_FILTER_CUSTOM_H */
