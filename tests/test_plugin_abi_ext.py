"""The rest of the public sub-plugin ABI (include/nnsx/):

* tensor_trainer frameworks in C (nnsx_plugin_api_trainer.h; reference
  nnstreamer_plugin_api_trainer.h:31-141): create / start / push_data /
  getFrameworkInfo / destroy, the epoch + training-complete notifications that
  replace the reference's GCond, model save;
* the seven V1 filter events (nnstreamer_plugin_api_filter.h:199-262):
  CUSTOM_PROP, SET_INPUT_PROP, SET_OUTPUT_PROP, SET_ACCELERATOR,
  CHECK_HW_AVAILABILITY, DESTROY_NOTIFY (+ RELOAD_MODEL, covered elsewhere);
* the legacy V0 table (invoke_NN / get*Dimension / setInputDimension / ...);
* the C++ framework base nnsx::tensor_filter_subplugin
  (nnstreamer_cppplugin_api_filter.hh:67-198) and framework=cpp objects
  nnsx::tensor_filter_cpp (tensor_filter_cpp.hh), each built as an external
  shared object with the system compiler against the installed headers.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
F4 = "other/tensors,format=static,num_tensors=1,dimensions=4,types=float32,framerate=0/1"

TRAINER_SRC = r"""
#include <nnsx/nnsx_plugin_api.h>
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* a "model" that tracks the mean of input[0] per epoch: training loss = that
   mean, accuracy = samples / expected; saves the epoch count on completion */
typedef struct { long seen, epoch; double sum, vsum; long nt, nv; double loss, vloss; int done, started; } st_t;
int ctrain_destroyed = 0;

static int t_create(const NNSX_TrainerFramework *self, const NNSX_TrainerProperties *p, void **pd) {
  (void)self;
  if (p->num_inputs != 1 || p->num_labels != 1) return -EINVAL;
  *pd = calloc(1, sizeof(st_t));
  return 0;
}
static int t_destroy(const NNSX_TrainerFramework *self, const NNSX_TrainerProperties *p, void **pd) {
  (void)self; (void)p; free(*pd); *pd = NULL; ++ctrain_destroyed; return 0;
}
static int t_start(const NNSX_TrainerFramework *self, const NNSX_TrainerProperties *p, void *pd) {
  (void)self; (void)p; ((st_t *)pd)->started = 1; return 0;
}
static int t_push(const NNSX_TrainerFramework *self, const NNSX_TrainerProperties *p, void *pd,
                  const NNSX_TensorMemory *in) {
  st_t *s = (st_t *)pd;
  (void)self;
  if (!s->started || s->done) return -EINVAL;
  const float *x = (const float *)in[0].data;
  const long per = p->num_training_samples + p->num_validation_samples;
  const long k = s->seen % per;
  if (k < p->num_training_samples) { s->sum += x[0]; s->nt++; } else { s->vsum += x[0]; s->nv++; }
  s->seen++;
  if (s->seen % per == 0) {
    s->loss = s->sum / s->nt; s->vloss = s->nv ? s->vsum / s->nv : 0;
    s->sum = s->vsum = 0; s->nt = s->nv = 0;
    s->epoch++;
    p->notify(p->notify_handle, NNSX_TRAINER_EVENT_EPOCH_COMPLETION);
    if (s->epoch == p->num_epochs) {
      FILE *f = fopen(p->model_save_path, "w");
      if (f) { fprintf(f, "epochs=%ld\n", s->epoch); fclose(f); }
      s->done = 1;
      p->notify(p->notify_handle, NNSX_TRAINER_EVENT_TRAINING_COMPLETION);
    }
  }
  return 0;
}
static int t_info(const NNSX_TrainerFramework *self, const NNSX_TrainerProperties *p, void *pd,
                  NNSX_TrainerFrameworkInfo *i) {
  (void)self; (void)p;
  memset(i, 0, sizeof(*i));
  i->name = "ctrain";
  if (!pd) return 0;
  const st_t *s = (const st_t *)pd;
  i->is_training_complete = s->done; i->epoch_cnt = s->epoch;
  i->training_loss = s->loss; i->validation_loss = s->vloss;
  i->training_accuracy = 1.0; i->validation_accuracy = 0.5;
  return 0;
}
static NNSX_TrainerFramework tfw = {NNSX_TRAINER_FRAMEWORK_V1, "ctrain", t_create, t_destroy, t_start, NULL, t_push,
                                    t_info, NULL};
int nnsx_subplugin_init(const NNSX_PluginHost *host) {
  if (host->abi_version < 2) return -EINVAL;
  return host->register_trainer(&tfw);
}
"""

EVENTS_SRC = r"""
#include <nnsx/nnsx_plugin_api.h>
#include <errno.h>
#include <stdlib.h>
#include <string.h>

/* y = k * x with allocate-in-invoke outputs freed through DESTROY_NOTIFY; the
   events it saw are recorded for the test (read back with ctypes) */
char evlog[512] = "";
int freed = 0;
typedef struct { float k; } priv_t;
static void logev(const char *s) { strncat(evlog, s, sizeof(evlog) - strlen(evlog) - 1); strncat(evlog, ";", 2); }
static float parse_k(const char *c) { const char *p = c ? strstr(c, "k:") : NULL; return p ? (float)atof(p + 2) : 1.0f; }

static int e_open(const NNSX_FilterProperties *prop, void **pd) {
  priv_t *p = (priv_t *)calloc(1, sizeof(priv_t));
  p->k = parse_k(prop->custom_properties);
  *pd = p;
  return 0;
}
static void e_close(const NNSX_FilterProperties *prop, void **pd) { (void)prop; free(*pd); *pd = NULL; }
static int e_info(const NNSX_FilterFramework *self, const NNSX_FilterProperties *prop, void *pd, NNSX_FrameworkInfo *i) {
  (void)self; (void)prop; (void)pd;
  memset(i, 0, sizeof(*i));
  i->name = "cevents"; i->allocate_in_invoke = 1; i->run_without_model = 1; i->accelerators = "cpu,gpu";
  return 0;
}
static int e_model(const NNSX_FilterFramework *self, const NNSX_FilterProperties *prop, void *pd, NNSX_ModelInfoOps op,
                   NNSX_TensorsInfo *in, NNSX_TensorsInfo *out) {
  (void)self; (void)prop; (void)pd;
  if (op != NNSX_SET_INPUT_INFO) return -ENOENT;
  *out = *in;
  return 0;
}
static int e_invoke(const NNSX_FilterFramework *self, const NNSX_FilterProperties *prop, void *pd,
                    const NNSX_TensorMemory *in, NNSX_TensorMemory *out, const NNSX_InvokeContext *ctx) {
  (void)self; (void)prop; (void)ctx;
  const priv_t *p = (const priv_t *)pd;
  out[0].data = malloc(in[0].size);
  out[0].size = in[0].size;
  for (size_t i = 0; i < in[0].size / 4; ++i) ((float *)out[0].data)[i] = p->k * ((const float *)in[0].data)[i];
  return 0;
}
static int e_event(const NNSX_FilterFramework *self, const NNSX_FilterProperties *prop, void *pd, NNSX_FilterEvent ev,
                   const void *data) {
  const NNSX_FilterEventData *d = (const NNSX_FilterEventData *)data;
  (void)self; (void)prop;
  switch (ev) {
    case NNSX_EVENT_CUSTOM_PROP: ((priv_t *)pd)->k = parse_k(d->custom_properties); logev("custom"); return 0;
    case NNSX_EVENT_SET_INPUT_PROP: logev(d->info->num_tensors == 1 ? "input1" : "input?"); return 0;
    case NNSX_EVENT_SET_OUTPUT_PROP: logev("output"); return 0;
    case NNSX_EVENT_SET_ACCELERATOR: logev("accel"); logev(d->accelerators); return 0;
    case NNSX_EVENT_CHECK_HW_AVAILABILITY: logev("hw"); logev(d->hw); return strcmp(d->hw, "cpu") == 0 ? 0 : -ENODEV;
    case NNSX_EVENT_DESTROY_NOTIFY: free(d->data); ++freed; return 0;
    default: return -ENOENT;
  }
}
static NNSX_FilterFramework fw = {NNSX_FILTER_FRAMEWORK_V1, "cevents", e_open, e_close, e_info, e_model, e_invoke,
                                  NULL, e_event, NULL};
int nnsx_subplugin_init(const NNSX_PluginHost *host) { return host->register_filter(&fw); }
"""

V0_SRC = r"""
#include <nnsx/nnsx_plugin_api.h>
#include <errno.h>
#include <stdlib.h>
#include <string.h>

/* V0 table: fixed 4 -> 2 (pairwise sums), invoke allocates */
int v0_reloads = 0;
static int o(const NNSX_FilterProperties *p, void **pd) { (void)p; *pd = malloc(1); return 0; }
static void c(const NNSX_FilterProperties *p, void **pd) { (void)p; free(*pd); *pd = NULL; }
static int inv(const NNSX_FilterProperties *p, void **pd, const NNSX_TensorMemory *in, NNSX_TensorMemory *out) {
  (void)p; (void)pd;
  const float *x = (const float *)in[0].data;
  float *y = (float *)malloc(8);
  y[0] = x[0] + x[1]; y[1] = x[2] + x[3];
  out[0].data = y; out[0].size = 8;
  return 0;
}
static void fill(NNSX_TensorsInfo *i, unsigned n) {
  memset(i, 0, sizeof(*i)); i->num_tensors = 1; i->info[0].type = 7; i->info[0].dimension[0] = n;
  for (int d = 1; d < 8; ++d) i->info[0].dimension[d] = 1;
}
static int gin(const NNSX_FilterProperties *p, void **pd, NNSX_TensorsInfo *i) { (void)p; (void)pd; fill(i, 4); return 0; }
static int gout(const NNSX_FilterProperties *p, void **pd, NNSX_TensorsInfo *i) { (void)p; (void)pd; fill(i, 2); return 0; }
static int avail(const char *hw) { return strcmp(hw, "cpu") == 0 ? 0 : -ENODEV; }
static int alloc_ii(void **pd) { (void)pd; return 0; }
static NNSX_FilterFrameworkV0 v0 = {NNSX_FILTER_FRAMEWORK_V0, "cpairsum", 0, 1, 1, 0, o, c, inv, gin, gout, NULL,
                                    NULL, NULL, NULL, avail, alloc_ii};
int nnsx_subplugin_init(const NNSX_PluginHost *host) {
  return host->register_filter((const NNSX_FilterFramework *)&v0);
}
"""

CPP_SUBPLUGIN_SRC = r"""
#include <nnsx/nnsx_cppplugin_api_filter.hh>
#include <cstring>
#include <stdexcept>
#include <string>

// y = x + offset (custom=off:<v>), as a class on the C++ framework base
class cpp_offset : public nnsx::tensor_filter_subplugin {
 public:
  tensor_filter_subplugin &getEmptyInstance() override { return *new cpp_offset(); }
  void configure_instance(const NNSX_FilterProperties *prop) override {
    const char *c = prop->custom_properties ? std::strstr(prop->custom_properties, "off:") : nullptr;
    off_ = c ? std::stof(c + 4) : 0.f;
    if (off_ < -1000) throw std::invalid_argument("offset out of range");
  }
  void invoke(const NNSX_TensorMemory *in, NNSX_TensorMemory *out) override {
    for (size_t i = 0; i < in[0].size / 4; ++i)
      static_cast<float *>(out[0].data)[i] = static_cast<const float *>(in[0].data)[i] + off_;
  }
  void getFrameworkInfo(NNSX_FrameworkInfo &info) override {
    std::memset(&info, 0, sizeof(info));
    info.name = "cppoffset";
    info.run_without_model = 1;
    info.accelerators = "cpu";
  }
  int getModelInfo(NNSX_ModelInfoOps ops, NNSX_TensorsInfo &in, NNSX_TensorsInfo &out) override {
    if (ops != NNSX_SET_INPUT_INFO) return -ENOENT;
    out = in;
    return 0;
  }
 private:
  float off_ = 0.f;
};

static cpp_offset *reg = nullptr;
extern "C" int nnsx_subplugin_init(const NNSX_PluginHost *host) {
  reg = nnsx::tensor_filter_subplugin::register_subplugin<cpp_offset>(host);
  return reg ? 0 : -1;
}
"""

CPP_FILTER_SRC = r"""
#include <nnsx/tensor_filter_cpp.hh>
#include <cstdlib>
#include <cstring>

// framework=cpp object: 3 floats -> their reversed order, outputs allocated by the object
class reverser : public nnsx::tensor_filter_cpp {
 public:
  reverser() : tensor_filter_cpp("reverser01") {}
  int getInputDim(NNSX_TensorsInfo *info) override { fill(info); return 0; }
  int getOutputDim(NNSX_TensorsInfo *info) override { fill(info); return 0; }
  int setInputDim(const NNSX_TensorsInfo *, NNSX_TensorsInfo *) override { return -EINVAL; }
  bool isAllocatedBeforeInvoke() override { return false; }
  int invoke(const NNSX_TensorMemory *in, NNSX_TensorMemory *out) override {
    const float *x = static_cast<const float *>(in[0].data);
    float *y = static_cast<float *>(std::malloc(12));
    y[0] = x[2]; y[1] = x[1]; y[2] = x[0];
    out[0].data = y;
    out[0].size = 12;
    return 0;
  }
 private:
  static void fill(NNSX_TensorsInfo *i) {
    std::memset(i, 0, sizeof(*i));
    i->num_tensors = 1;
    i->info[0].type = 7;
    for (int d = 0; d < 8; ++d) i->info[0].dimension[d] = d == 0 ? 3 : 1;
  }
};

extern "C" int nnsx_subplugin_init(const NNSX_PluginHost *host) {
  static reverser r;
  return r._register(host);
}
"""


def _build(tmp, name, src, cxx=False):
    ext = ".cc" if cxx else ".c"
    f = tmp / (name + ext)
    f.write_text(src)
    so = tmp / ("lib" + name + ".so")
    cc = ["g++", "-std=c++14"] if cxx else ["gcc"]
    subprocess.run(cc + ["-shared", "-fPIC", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(f),
                         "-o", str(so)], check=True)
    return so


@pytest.fixture(scope="module")
def plugs(tmp_path_factory):
    d = tmp_path_factory.mktemp("abi_ext")
    libs = dict(trainer=_build(d, "nnstreamer_trainer_ctrain", TRAINER_SRC),
                events=_build(d, "nnstreamer_filter_cevents", EVENTS_SRC),
                v0=_build(d, "nnstreamer_filter_cpairsum", V0_SRC),
                cppsub=_build(d, "nnstreamer_filter_cppoffset", CPP_SUBPLUGIN_SRC, cxx=True),
                cppobj=_build(d, "reverser_objs", CPP_FILTER_SRC, cxx=True))
    keys = ("NNSTREAMER_FILTERS", "NNSTREAMER_TRAINERS")
    old = {k: os.environ.get(k) for k in keys}
    for k in keys:
        os.environ[k] = str(d)
    yield libs
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


def _run(nns, tail, frames, caps=F4, sink="sink", between=None):
    import time

    p = nns.parse_launch(f"appsrc name=src caps={caps} ! {tail}")
    out = []
    p.get_by_name(sink).connect("new-data", lambda b: out.append(b.memory(0).numpy("float32").copy()))
    p.set_state("playing")
    for i, f in enumerate(frames):
        if between:
            t = time.time()
            while len(out) < i and time.time() - t < 10:  # the earlier frames are through
                time.sleep(0.005)
            between(p, i)
        p.get_by_name("src").push_buffer(f, pts=i)
    p.get_by_name("src").end_of_stream()
    assert p.wait(30)[0] == "eos", p.messages()
    return p, out


def test_external_c_trainer(nns, plugs, tmp_path):
    save = tmp_path / "ctrain.model"
    caps = "other/tensors,format=static,num_tensors=2,dimensions=4.1,types=float32.float32,framerate=0/1"
    p = nns.parse_launch(
        f"appsrc name=src caps={caps} ! tensor_trainer name=tr framework=ctrain model-config=none "
        f"model-save-path={save} num-inputs=1 num-labels=1 num-training-samples=3 num-validation-samples=1 "
        "epochs=2 ! tensor_sink name=sink")
    stats = []
    p.get_by_name("sink").connect("new-data", lambda b: stats.append(b.memory(0).numpy("float64").copy()))
    p.set_state("playing")
    vals = [1, 2, 3, 10, 4, 5, 6, 20]  # epoch 0: train mean 2, val 10; epoch 1: train mean 5, val 20
    for i, v in enumerate(vals):
        p.get_by_name("src").push_buffer([np.full(4, v, np.float32), np.zeros(1, np.float32)], pts=i)
    p.get_by_name("src").end_of_stream()
    assert p.wait(30)[0] == "eos", p.messages()
    assert int(p.get_by_name("tr").get_property("epoch-count")) == 2
    p.stop()
    assert len(stats) == 3  # first sample + two epoch ends
    np.testing.assert_allclose(stats[1], [2, 1, 10, 0.5])
    np.testing.assert_allclose(stats[2], [5, 1, 20, 0.5])
    assert save.read_text() == "epochs=2\n"
    lib = ctypes.CDLL(str(plugs["trainer"]))
    assert ctypes.c_int.in_dll(lib, "ctrain_destroyed").value == 1


def test_v1_filter_events(nns, plugs):
    lib = ctypes.CDLL(str(plugs["events"]))
    frames = [np.array([1, 2, 3, 4], np.float32)] * 4

    def change(p, i):
        f = p.get_by_name("f")
        if i == 2:
            f.set_property("custom", "k:5")            # CUSTOM_PROP
            f.set_property("inputtype", "float32")
            f.set_property("input", "4")               # SET_INPUT_PROP
            f.set_property("accelerator", "true:cpu")  # SET_ACCELERATOR

    p, out = _run(nns, "tensor_filter name=f framework=cevents custom=k:2 ! tensor_sink name=sink", frames,
                  between=change)
    p.stop()
    np.testing.assert_array_equal(out[0], [2, 4, 6, 8])
    np.testing.assert_array_equal(out[3], [5, 10, 15, 20])
    log = ctypes.c_char_p.in_dll(lib, "evlog")  # noqa: F841 (char array: read below)
    text = ctypes.string_at(ctypes.addressof(ctypes.c_char.in_dll(lib, "evlog"))).decode()
    assert "custom;" in text and "input1;" in text and "accel;" in text, text
    # allocate-in-invoke outputs came back through DESTROY_NOTIFY (handled: freed by the plugin)
    assert ctypes.c_int.in_dll(lib, "freed").value == 4


def test_check_hw_availability_event(nns, plugs):
    lib = ctypes.CDLL(str(plugs["events"]))
    # the table advertises gpu, but the CHECK_HW_AVAILABILITY answer decides
    p = nns.parse_launch(f"appsrc name=src caps={F4} ! tensor_filter framework=cevents accelerator=true:gpu "
                         "! tensor_sink name=sink")
    p.set_state("playing")
    p.get_by_name("src").push_buffer(np.ones(4, np.float32), pts=0)
    p.get_by_name("src").end_of_stream()
    msg = p.wait(30)
    p.stop()
    text = ctypes.string_at(ctypes.addressof(ctypes.c_char.in_dll(lib, "evlog"))).decode()
    assert "hw;gpu;" in text, text
    assert msg is not None


def test_v0_table(nns, plugs):
    p, out = _run(nns, "tensor_filter framework=cpairsum ! tensor_sink name=sink",
                  [np.array([1, 2, 3, 4], np.float32), np.array([0.5, 0.5, -1, 1], np.float32)])
    p.stop()
    np.testing.assert_array_equal(out[0], [3, 7])
    np.testing.assert_array_equal(out[1], [1, 0])


def test_cpp_subplugin_base(nns, plugs):
    p, out = _run(nns, "tensor_filter framework=cppoffset custom=off:1.5 ! tensor_sink name=sink",
                  [np.array([1, 2, 3, 4], np.float32)])
    p.stop()
    np.testing.assert_array_equal(out[0], [2.5, 3.5, 4.5, 5.5])
    # a configure_instance exception is an open failure, not a crash
    p = nns.parse_launch(f"appsrc name=src caps={F4} ! tensor_filter framework=cppoffset custom=off:-5000 "
                         "! tensor_sink name=sink")
    p.set_state("playing")
    p.get_by_name("src").push_buffer(np.ones(4, np.float32), pts=0)
    msg = p.wait(20)
    p.stop()
    assert msg and msg[0] == "error"


def test_framework_cpp_object_from_library(nns, plugs):
    caps = "other/tensors,format=static,num_tensors=1,dimensions=3,types=float32,framerate=0/1"
    # the reference's model order: <name>,<library>
    p, out = _run(nns, f"tensor_filter framework=cpp model=reverser01,{plugs['cppobj']} ! tensor_sink name=sink",
                  [np.array([1, 2, 3], np.float32)], caps=caps)
    p.stop()
    np.testing.assert_array_equal(out[0], [3, 2, 1])
