/*
 * nnsx public sub-plugin ABI: external tensor_filter frameworks, tensor_decoder
 * modes and tensor_converter converters as plain-C shared objects.
 *
 * Counterpart of NNStreamer's nnstreamer_plugin_api_{filter,decoder,converter}.h
 * (GstTensorFilterFramework V1, GstTensorDecoderDef, NNStreamerExternalConverter)
 * without GLib/GStreamer types: caps travel as strings, tensors as the plain
 * structs of tensor_filter_custom.h, and a filter invoke receives the GPU it
 * runs on and the HIP stream of its element (device-resident memories).
 *
 * Loading: a sub-plugin is a shared object named
 *   libnnstreamer_filter_<name>.so / libnnstreamer_decoder_<name>.so /
 *   libnnstreamer_converter_<name>.so / libnnstreamer_trainer_<name>.so
 * in a sub-plugin directory (ini [filter]/[decoder]/[converter]/[trainer]
 * paths, NNSTREAMER_FILTERS / _DECODERS / _CONVERTERS / _TRAINERS,
 * NNSX_SUBPLUGIN_PATH).  On the
 * first lookup of <name> the runtime dlopen()s it and calls its exported
 *
 *   int nnsx_subplugin_init(const NNSX_PluginHost *host);
 *
 * which registers its tables through host->register_*(), the way the
 * reference's sub-plugins call nnstreamer_filter_probe() from a constructor.
 * The host table is the only link to the runtime, so a sub-plugin needs no
 * link-time dependency on it (the runtime library may be loaded RTLD_LOCAL,
 * e.g. as a Python extension).  Tables must stay valid until
 * host->unregister_*() or process exit.
 *
 * Return codes: 0 = success, negative = error (-errno style); a filter invoke
 * returning > 0 drops the frame.
 */
#ifndef NNSX_PLUGIN_API_H
#define NNSX_PLUGIN_API_H

#include <nnsx/nnstreamer_custom.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: register_trainer / unregister_trainer and register_cpp_filter /
 * unregister_cpp_filter appended to the host table.  A sub-plugin checks
 * host->abi_version >= the version whose entries it uses. */
#define NNSX_PLUGIN_ABI_VERSION 2u

typedef struct _NNSX_FilterFramework NNSX_FilterFramework;
typedef struct _NNSX_Decoder NNSX_Decoder;
typedef struct _NNSX_Converter NNSX_Converter;
typedef struct _NNSX_TrainerFramework NNSX_TrainerFramework;

typedef struct {
  uint32_t abi_version; /* NNSX_PLUGIN_ABI_VERSION */
  int (*register_filter)(const NNSX_FilterFramework *fw);
  int (*unregister_filter)(const char *name);
  int (*register_decoder)(const NNSX_Decoder *dec);
  int (*unregister_decoder)(const char *modename);
  int (*register_converter)(const NNSX_Converter *conv);
  int (*unregister_converter)(const char *name);
  /* level: 0 error, 1 warning, 2 info, 3 debug */
  void (*log)(int level, const char *category, const char *message);
  /* abi_version >= 2 */
  int (*register_trainer)(const NNSX_TrainerFramework *fw);
  int (*unregister_trainer)(const char *name);
  /* framework=cpp objects; ops: NNSX_CppFilterOps of <nnsx/nnsx_plugin_api_filter.h> */
  int (*register_cpp_filter)(const char *name, void *obj, const void *ops);
  int (*unregister_cpp_filter)(const char *name);
} NNSX_PluginHost;

/* exported by every sub-plugin shared object */
typedef int (*NNSX_SubpluginInitFunc)(const NNSX_PluginHost *host);
#define NNSX_SUBPLUGIN_INIT_SYMBOL "nnsx_subplugin_init"

/* The same registration entry points, exported by the runtime for in-process
 * use (applications linked against it): reference names. */
int nnstreamer_filter_probe(const NNSX_FilterFramework *fw);
int nnstreamer_filter_exit(const char *name);
int nnstreamer_decoder_probe(const NNSX_Decoder *dec);
int nnstreamer_decoder_exit(const char *modename);
int registerExternalConverter(const NNSX_Converter *conv);
int unregisterExternalConverter(const char *name);
int nnstreamer_cpp_filter_register(const char *name, void *obj, const void *ops);
int nnstreamer_cpp_filter_unregister(const char *name);

#ifdef __cplusplus
}
#endif

#include <nnsx/nnsx_plugin_api_filter.h>
#include <nnsx/nnsx_plugin_api_decoder.h>
#include <nnsx/nnsx_plugin_api_converter.h>
#include <nnsx/nnsx_plugin_api_trainer.h>

#endif /* NNSX_PLUGIN_API_H */
