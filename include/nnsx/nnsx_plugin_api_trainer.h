/*
 * nnsx tensor_trainer framework ABI.  Reference:
 * gst/nnstreamer/include/nnstreamer_plugin_api_trainer.h:31-141
 * (GstTensorTrainerProperties, GstTensorTrainerFrameworkInfo,
 * GstTensorTrainerFramework: create / destroy / start / push_data /
 * getFrameworkInfo; nnstreamer_trainer_probe / nnstreamer_trainer_exit).
 * Include <nnsx/nnsx_plugin_api.h>.
 *
 * The reference hands the sub-plugin a GCond it signals when training is
 * complete; without GLib the properties carry a notify callback instead:
 *   prop->notify(prop->notify_handle, NNSX_TRAINER_EVENT_TRAINING_COMPLETION)
 * after the last epoch (tensor_trainer waits for it at EOS), and
 *   prop->notify(prop->notify_handle, NNSX_TRAINER_EVENT_EPOCH_COMPLETION)
 * after each epoch (tensor_trainer then reads getFrameworkInfo and pushes the
 * [training loss, training accuracy, validation loss, validation accuracy]
 * tensor downstream).  The callback may be called from any thread.
 *
 * Samples: tensor_trainer calls push_data once per incoming buffer with its
 * num_inputs + num_labels tensors (host memory); per epoch the first
 * num_training_samples are training samples, the next num_validation_samples
 * validation samples, for num_epochs epochs (the reference's counting).
 */
#ifndef NNSX_PLUGIN_API_TRAINER_H
#define NNSX_PLUGIN_API_TRAINER_H

#include <nnsx/nnstreamer_custom.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NNSX_TRAINER_FRAMEWORK_V1 0x4e545231u /* 'NTR1' */

typedef enum {
  NNSX_TRAINER_EVENT_EPOCH_COMPLETION = 0,
  NNSX_TRAINER_EVENT_TRAINING_COMPLETION = 1,
} NNSX_TrainerEvent;

typedef struct {
  NNSX_TensorsInfo input_meta; /* configured input tensors (inputs then labels) */
  const char *model_config;    /* model-config: the configuration file creating the model */
  const char *model_save_path; /* model-save-path: where the trained model is saved */
  const char *model_load_path; /* model-load-path: an existing model to continue from (may be NULL) */
  int64_t num_inputs;
  int64_t num_labels;
  int64_t num_training_samples;
  int64_t num_validation_samples;
  int64_t num_epochs;
  int device; /* nnsx: GPU the trainer may use, -1 = CPU */
  void (*notify)(void *notify_handle, NNSX_TrainerEvent event);
  void *notify_handle;
} NNSX_TrainerProperties;

typedef struct {
  const char *name;         /* searchable by tensor_trainer framework= */
  int is_training_complete; /* nonzero once every epoch ran */
  int64_t epoch_cnt;        /* completed epochs */
  /* nnsx: the statistics tensor_trainer emits after each epoch */
  double training_loss, training_accuracy, validation_loss, validation_accuracy;
} NNSX_TrainerFrameworkInfo;

typedef struct _NNSX_TrainerFramework NNSX_TrainerFramework;
struct _NNSX_TrainerFramework {
  uint32_t version; /* NNSX_TRAINER_FRAMEWORK_V1 */
  const char *name;
  /* create the model; store per-instance state in *private_data */
  int (*create)(const NNSX_TrainerFramework *self, const NNSX_TrainerProperties *prop, void **private_data);
  /* destroy it; set *private_data = NULL */
  int (*destroy)(const NNSX_TrainerFramework *self, const NNSX_TrainerProperties *prop, void **private_data);
  /* start training (samples follow through push_data) */
  int (*start)(const NNSX_TrainerFramework *self, const NNSX_TrainerProperties *prop, void *private_data);
  /* optional (nnsx): stop early (pipeline stop / flush); NULL = nothing to do */
  int (*stop)(const NNSX_TrainerFramework *self, const NNSX_TrainerProperties *prop, void *private_data);
  /* one sample: num_inputs + num_labels tensors */
  int (*push_data)(const NNSX_TrainerFramework *self, const NNSX_TrainerProperties *prop, void *private_data,
                   const NNSX_TensorMemory *input);
  /* mandatory; private_data is NULL when asked before create */
  int (*getFrameworkInfo)(const NNSX_TrainerFramework *self, const NNSX_TrainerProperties *prop, void *private_data,
                          NNSX_TrainerFrameworkInfo *fw_info);
  /* optional (nnsx): save the model to `path` now (0 = saved) */
  int (*save)(const NNSX_TrainerFramework *self, const NNSX_TrainerProperties *prop, void *private_data,
              const char *path);
};

/* reference-named in-process registration (exported by the runtime) */
int nnstreamer_trainer_probe(const NNSX_TrainerFramework *ttsp);
int nnstreamer_trainer_exit(const char *name);

#ifdef __cplusplus
}
#endif

#endif /* NNSX_PLUGIN_API_TRAINER_H */
