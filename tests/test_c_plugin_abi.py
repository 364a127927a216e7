"""Public C sub-plugin ABI (include/nnsx/nnsx_plugin_api*.h): a tensor_filter
framework, a tensor_decoder mode and a tensor_converter converter, each built
from C as libnnstreamer_<kind>_<name>.so in a sub-plugin directory, found by
the registry's dlopen lookup and registered through nnsx_subplugin_init()
(reference flow: nnstreamer_subplugin.c:108-171, tables of
nnstreamer_plugin_api_filter.h:273-495, _decoder.h:38-97, _converter.h:41-85)."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

FILTER_SRC = r"""
#include <nnsx/nnsx_plugin_api.h>
#include <errno.h>
#include <stdlib.h>
#include <string.h>

typedef struct { float k; int closed; } priv_t;
static int opened = 0;

static int f_open(const NNSX_FilterProperties *prop, void **pd) {
  priv_t *p = (priv_t *)calloc(1, sizeof(priv_t));
  /* custom=k:<factor> */
  const char *c = prop->custom_properties ? strstr(prop->custom_properties, "k:") : NULL;
  p->k = c ? (float)atof(c + 2) : 2.0f;
  *pd = p;
  ++opened;
  return 0;
}
static void f_close(const NNSX_FilterProperties *prop, void **pd) { (void)prop; free(*pd); *pd = NULL; }
static int f_info(const NNSX_FilterFramework *self, const NNSX_FilterProperties *prop, void *pd, NNSX_FrameworkInfo *i) {
  (void)self; (void)prop; (void)pd;
  memset(i, 0, sizeof(*i));
  i->name = "cscale"; i->allocate_in_invoke = 0; i->run_without_model = 1; i->verify_model_path = 0;
  i->accelerators = "cpu"; i->model_extensions = ".cscale";
  return 0;
}
static int f_model(const NNSX_FilterFramework *self, const NNSX_FilterProperties *prop, void *pd, NNSX_ModelInfoOps op,
                   NNSX_TensorsInfo *in, NNSX_TensorsInfo *out) {
  (void)self; (void)prop; (void)pd;
  if (op != NNSX_SET_INPUT_INFO) return -ENOENT;  /* shapes follow the input */
  *out = *in;
  return 0;
}
static int f_invoke(const NNSX_FilterFramework *self, const NNSX_FilterProperties *prop, void *pd,
                    const NNSX_TensorMemory *in, NNSX_TensorMemory *out, const NNSX_InvokeContext *ctx) {
  const priv_t *p = (const priv_t *)pd;
  (void)self; (void)prop;
  if (ctx->device != -1 || out[0].size != in[0].size) return -EINVAL;
  for (size_t i = 0; i < in[0].size / 4; ++i) ((float *)out[0].data)[i] = p->k * ((const float *)in[0].data)[i];
  return 0;
}
static NNSX_FilterFramework fw = {NNSX_FILTER_FRAMEWORK_V1, "cscale", f_open, f_close, f_info, f_model, f_invoke,
                                  NULL, NULL};

int nnsx_subplugin_init(const NNSX_PluginHost *host) {
  if (host->abi_version < 1) return -EINVAL;
  host->log(2, "cscale", "registering framework cscale");
  return host->register_filter(&fw);
}
"""

DECODER_SRC = r"""
#include <nnsx/nnsx_plugin_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int d_init(void **pd) { *pd = calloc(1, 64); strcpy((char *)*pd, "sum"); return 0; }
static void d_exit(void **pd) { free(*pd); *pd = NULL; }
static int d_opt(void **pd, int op, const char *param) { if (op == 0) snprintf((char *)*pd, 64, "%s", param); return 0; }
static char *d_caps(void **pd, const NNSX_TensorsConfig *c) {
  (void)pd; (void)c;
  return strdup("text/x-raw, format=(string)utf8");
}
static size_t d_size(void **pd, const NNSX_TensorsConfig *c, size_t in) { (void)pd; (void)c; (void)in; return 64; }
static int d_decode(void **pd, const NNSX_TensorsConfig *c, const NNSX_TensorMemory *in, NNSX_TensorMemory *out) {
  double s = 0;
  for (size_t i = 0; i < in[0].size / 4; ++i) s += ((const float *)in[0].data)[i];
  out->size = (size_t)snprintf((char *)out->data, 64, "%s=%g/%u", (const char *)*pd, s, c->info.num_tensors);
  return 0;
}
static NNSX_Decoder dec = {"csum", d_init, d_exit, d_opt, d_caps, d_decode, d_size};
int nnsx_subplugin_init(const NNSX_PluginHost *host) { return host->register_decoder(&dec); }
"""

CONVERTER_SRC = r"""
#include <nnsx/nnsx_plugin_api.h>
#include <stdlib.h>
#include <string.h>

static char *c_caps(void) { return strdup("application/x-nnsx-cbytes"); }
/* every byte b -> float32 (b * 0.5) */
static int c_convert(const NNSX_TensorMemory *in, NNSX_TensorsConfig *cfg, NNSX_TensorMemory *out) {
  memset(cfg, 0, sizeof(*cfg));
  cfg->info.num_tensors = 1;
  cfg->info.info[0].type = 7; /* float32 */
  cfg->info.info[0].dimension[0] = (uint32_t)in->size;
  cfg->rate_n = 0; cfg->rate_d = 1;
  float *y = (float *)malloc(in->size * 4);
  for (size_t i = 0; i < in->size; ++i) y[i] = 0.5f * ((const unsigned char *)in->data)[i];
  out[0].data = y;
  out[0].size = in->size * 4;
  return 0;
}
static NNSX_Converter conv = {"cbytes", c_caps, NULL, c_convert};
int nnsx_subplugin_init(const NNSX_PluginHost *host) { return host->register_converter(&conv); }
"""


def _build(tmp, name, src):
    c = tmp / (name + ".c")
    c.write_text(src)
    so = tmp / ("lib" + name + ".so")
    subprocess.run(["gcc", "-shared", "-fPIC", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(c),
                    "-o", str(so)], check=True)
    return so


@pytest.fixture(scope="module")
def plugdir(tmp_path_factory):
    d = tmp_path_factory.mktemp("subplugins")
    _build(d, "nnstreamer_filter_cscale", FILTER_SRC)
    _build(d, "nnstreamer_decoder_csum", DECODER_SRC)
    _build(d, "nnstreamer_converter_cbytes", CONVERTER_SRC)
    old = {k: os.environ.get(k) for k in ("NNSTREAMER_FILTERS", "NNSTREAMER_DECODERS", "NNSTREAMER_CONVERTERS")}
    os.environ["NNSTREAMER_FILTERS"] = str(d)
    os.environ["NNSTREAMER_DECODERS"] = str(d)
    os.environ["NNSTREAMER_CONVERTERS"] = str(d)
    yield d
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


def test_external_filter_and_decoder_from_c(nns, plugdir):
    caps = "other/tensors,format=static,num_tensors=1,dimensions=4,types=float32,framerate=0/1"
    p = nns.parse_launch(f"appsrc name=src caps={caps} ! tensor_filter framework=cscale custom=k:3 "
                         "! tee name=t t. ! queue ! tensor_decoder mode=csum option1=total ! tensor_sink name=txt "
                         "t. ! queue ! tensor_sink name=raw")
    texts, raw = [], []
    p.get_by_name("txt").connect("new-data", lambda b: texts.append(b.memory(0).bytes().decode()))
    p.get_by_name("raw").connect("new-data", lambda b: raw.append(b.memory(0).numpy("float32").copy()))
    p.set_state("playing")
    src = p.get_by_name("src")
    src.push_buffer(np.array([1, 2, 3, 4], np.float32), pts=0)
    src.push_buffer(np.array([0.5, 0, 0, 0], np.float32), pts=1)
    src.end_of_stream()
    assert p.wait(30)[0] == "eos", p.messages()
    p.stop()
    np.testing.assert_array_equal(raw[0], [3, 6, 9, 12])
    assert texts == ["total=30/1", "total=1.5/1"]


def test_external_converter_from_c_selected_by_caps(nns, plugdir):
    p = nns.parse_launch("appsrc name=src caps=application/x-nnsx-cbytes ! tensor_converter ! tensor_sink name=s")
    got = []
    p.get_by_name("s").connect("new-data", lambda b: got.append(b.memory(0).numpy("float32").copy()))
    p.set_state("playing")
    p.get_by_name("src").push_buffer(np.array([2, 4, 255], np.uint8), pts=0)
    p.get_by_name("src").end_of_stream()
    assert p.wait(30)[0] == "eos", p.messages()
    p.stop()
    np.testing.assert_array_equal(got[0], [1.0, 2.0, 127.5])


def test_framework_auto_detects_plugin_extension(nns, plugdir, tmp_path):
    # the C table's model_extensions drive framework=auto
    model = tmp_path / "m.cscale"
    model.write_text("x")
    caps = "other/tensors,format=static,num_tensors=1,dimensions=2,types=float32,framerate=0/1"
    p = nns.parse_launch(f"appsrc name=src caps={caps} ! tensor_filter framework=auto model={model} "
                         "! tensor_sink name=s")
    got = []
    p.get_by_name("s").connect("new-data", lambda b: got.append(b.memory(0).numpy("float32").copy()))
    p.set_state("playing")
    p.get_by_name("src").push_buffer(np.array([1, -1], np.float32), pts=0)
    p.get_by_name("src").end_of_stream()
    assert p.wait(30)[0] == "eos", p.messages()
    p.stop()
    np.testing.assert_array_equal(got[0], [2, -2])
    assert "cscale" in nns.subplugins("filter")
