/*
 * nnsx tensor_converter external-converter ABI.  Reference:
 * gst/nnstreamer/include/nnstreamer_plugin_api_converter.h:41-85
 * (NNStreamerExternalConverter: name, convert, get_out_config, query_caps).
 * Include <nnsx/nnsx_plugin_api.h>.
 */
#ifndef NNSX_PLUGIN_API_CONVERTER_H
#define NNSX_PLUGIN_API_CONVERTER_H

#include <nnsx/nnstreamer_custom.h>

#ifdef __cplusplus
extern "C" {
#endif

struct _NNSX_Converter {
  const char *name;
  /* media caps this converter accepts, as a malloc()ed caps string (freed by
   * the runtime); tensor_converter picks the converter whose caps intersect
   * its input caps */
  char *(*query_caps)(void);
  /* tensors config for these input caps; 0 on success (optional) */
  int (*get_out_config)(const char *in_caps, NNSX_TensorsConfig *config);
  /* one input buffer (host-mapped, all memories concatenated) -> fill *config
   * and out[0..config->info.num_tensors) with malloc()ed memories (freed by
   * the runtime) */
  int (*convert)(const NNSX_TensorMemory *in, NNSX_TensorsConfig *config, NNSX_TensorMemory *out);
};

#ifdef __cplusplus
}
#endif

#endif /* NNSX_PLUGIN_API_CONVERTER_H */
