/*
 * nnsx C API for in-process custom callbacks, with the reference's entry
 * point names:
 *
 *   NNS_custom_easy_register            (tensor_filter framework=custom-easy)
 *   nnstreamer_converter_custom_register (tensor_converter mode=custom-code:<name>)
 *   nnstreamer_decoder_custom_register   (tensor_decoder mode=custom-code option1=<name>)
 *   nnstreamer_if_custom_register        (tensor_if compared-value=CUSTOM)
 *
 * Reference: gst/nnstreamer/include/tensor_filter_custom_easy.h,
 * nnstreamer_plugin_api_converter.h, nnstreamer_plugin_api_decoder.h,
 * tensor_if.h.  GLib / GstBuffer types are replaced by the plain structs of
 * tensor_filter_custom.h; memories handed to callbacks are host-mapped.
 * Return values: 0 = success, negative = error.
 */
#ifndef NNSX_NNSTREAMER_CUSTOM_H
#define NNSX_NNSTREAMER_CUSTOM_H

#include <nnsx/tensor_filter_custom.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  NNSX_TensorsInfo info;
  int rate_n;
  int rate_d;
} NNSX_TensorsConfig;

/* custom-easy: outputs are pre-allocated per out_info; return 0 (pass), > 0 (drop the frame), < 0 (error) */
typedef int (*NNS_custom_easy_invoke)(void *data, const NNSX_FilterProperties *prop, const NNSX_TensorMemory *input,
                                      NNSX_TensorMemory *output);
int NNS_custom_easy_register(const char *modelname, NNS_custom_easy_invoke func, void *data,
                             const NNSX_TensorsInfo *in_info, const NNSX_TensorsInfo *out_info);
int NNS_custom_easy_unregister(const char *modelname);

/* converter: raw input bytes -> tensors.  Fill *config and out[0..num_tensors)
 * with malloc()ed memories (the framework frees them). */
typedef int (*tensor_converter_custom)(const void *in, size_t in_size, void *data, NNSX_TensorsConfig *config,
                                       NNSX_TensorMemory *out);
int nnstreamer_converter_custom_register(const char *name, tensor_converter_custom func, void *data);
int nnstreamer_converter_custom_unregister(const char *name);

/* decoder: tensors -> one output memory (malloc()ed, freed by the framework) */
typedef int (*tensor_decoder_custom)(const NNSX_TensorMemory *input, const NNSX_TensorsConfig *config, void *data,
                                     NNSX_TensorMemory *out);
int nnstreamer_decoder_custom_register(const char *name, tensor_decoder_custom func, void *data);
int nnstreamer_decoder_custom_unregister(const char *name);

/* tensor_if: *result = the condition; return 0 on success */
typedef int (*tensor_if_custom)(const NNSX_TensorsInfo *info, const NNSX_TensorMemory *input, void *data, int *result);
int nnstreamer_if_custom_register(const char *name, tensor_if_custom func, void *data);
int nnstreamer_if_custom_unregister(const char *name);

#ifdef __cplusplus
}
#endif

#endif /* NNSX_NNSTREAMER_CUSTOM_H */
