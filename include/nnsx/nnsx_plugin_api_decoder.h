/*
 * nnsx tensor_decoder sub-plugin ABI.  Reference:
 * gst/nnstreamer/include/nnstreamer_plugin_api_decoder.h:38-97
 * (GstTensorDecoderDef: modename, init, exit, setOption, getOutCaps, decode,
 * getTransformSize).  Include <nnsx/nnsx_plugin_api.h>.
 */
#ifndef NNSX_PLUGIN_API_DECODER_H
#define NNSX_PLUGIN_API_DECODER_H

#include <nnsx/nnstreamer_custom.h>

#ifdef __cplusplus
extern "C" {
#endif

struct _NNSX_Decoder {
  const char *modename; /* tensor_decoder mode=<modename> */
  int (*init)(void **private_data);
  void (*exit)(void **private_data);
  /* option1..option9 -> opNum 0..8 */
  int (*setOption)(void **private_data, int opNum, const char *param);
  /* output caps for this input config as a malloc()ed caps string (freed by
   * the runtime), or NULL if it cannot be decided yet */
  char *(*getOutCaps)(void **private_data, const NNSX_TensorsConfig *config);
  /* input: num_tensors host-mapped memories.  If getTransformSize is set the
   * runtime pre-allocates output->data with that many bytes; otherwise the
   * decoder sets output->data to a malloc()ed block (freed by the runtime). */
  int (*decode)(void **private_data, const NNSX_TensorsConfig *config, const NNSX_TensorMemory *input,
                NNSX_TensorMemory *output);
  /* optional */
  size_t (*getTransformSize)(void **private_data, const NNSX_TensorsConfig *config, size_t in_size);
};

#ifdef __cplusplus
}
#endif

#endif /* NNSX_PLUGIN_API_DECODER_H */
