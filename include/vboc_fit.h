/* vboc_fit.h - C ABI of the VBOC loop's NN fit on the device (vboc_amd/csrc/fit.hip -> libvboc_fit.so).
 *
 * Replaces the reference's training loops (plain pointers and sizes, device memory, HIP streams as void*):
 *   VBOC/triplependulum_vboc.py:415-466   model / Adam(lr) / MSELoss, the first fit
 *                                         (`while val > 1e-3 and it < it_max`, random.sample of 4096 rows)
 *   VBOC/triplependulum_vboc.py:526-556   the refits (2048 old + 2048 new rows per minibatch)
 *   VBOC/doublependulum_vboc.py:440-560, VBOC/pendulum_vboc.py:228-277 and the Cartesian main block: the same loop
 *   my_nn.py:20-34                        NeuralNetDIR (Linear-ReLU-Linear-ReLU-Linear-ReLU)
 * Supported (inputs, hidden, minibatch): inputs 6 with hidden 449..512, inputs 4 with 257..320, inputs 2 with
 * 65..128; minibatch a multiple of 32 up to 4096 (triple 6-500 / 4096, double and Cartesian 4-300 / 4096,
 * pendulum 2-100 / 64).  Other shapes return VBOC_FIT_EUNSUPPORTED (the caller trains them with PyTorch).
 */
#ifndef VBOC_FIT_H
#define VBOC_FIT_H

#ifdef __cplusplus
extern "C" {
#endif

#define VBOC_FIT_EARG (-1)
#define VBOC_FIT_EHIP (-2)
#define VBOC_FIT_EUNSUPPORTED (-3)

typedef struct vboc_fit* vboc_fit_handle;

/* A trainer: padded parameters, Adam moments (zero: torch.optim.Adam(model.parameters()) at :418), the sampler's
 * Philox stream (seed).  The moments and the Adam step count persist across fits, as the reference's one optimizer
 * object does. */
int vboc_fit_create(int inputs, int hidden, int minibatch, unsigned long long seed, vboc_fit_handle* out);
int vboc_fit_destroy(vboc_fit_handle h);

/* Parameters in torch's nn.Linear layouts (device float32): W0 [hidden][inputs], b0 [hidden], W1 [hidden][hidden],
 * b1 [hidden], W2 [1][hidden], b2 [1].  Ordered after the work already queued on `stream`; the copy is queued
 * before any later work on it. */
int vboc_fit_set_params(vboc_fit_handle h, const float* W0, const float* b0, const float* W1, const float* b1,
                        const float* W2, const float* b2, void* stream);
/* which: 0 the parameters, 1 Adam's exp_avg, 2 its exp_avg_sq (same layouts) */
int vboc_fit_get_params(vboc_fit_handle h, int which, float* W0, float* b0, float* W1, float* b1, float* W2,
                        float* b2, void* stream);

typedef struct {
  const float* F;        /* device float32 rows [n][ld]: the inputs, then the target |qdot| */
  long long n;           /* rows */
  long long n_new;       /* 0: first fit (minibatch = random.sample(range(n), k)); else the last n_new rows are
                            the new ones (k/2 from each part, :533-538) */
  int ld;                /* row stride in floats (>= inputs + 1) */
  long long it_max;      /* the loop runs while val > stop_val and it < it_max, it from 1 */
  double val0;           /* the loop's initial val: max of the targets, in float64 (:446) */
  double stop_val;       /* 1e-3 (pendulum 1e-4) */
  double beta;           /* EMA weight 0.95 (pendulum 0.8) */
  double lr;             /* Adam learning rate 1e-3 */
  int poll;              /* steps per HIP graph / per host poll of the stop flag */
  int graphs;            /* 1: replay a captured graph of `poll` steps; 0: launch the steps one by one */
  long long* iterations; /* out: it - 1 at the stop (the steps taken) */
  double* val;           /* out: val at the stop */
  long long* launched;   /* out: steps launched (a multiple of poll; the ones past the stop are no-ops) */
  double* kernel_ms;     /* out: device time of the fit on the trainer's stream */
} vboc_fit_run_t;

/* One fit: returns 0 when the loop stopped (val <= stop_val or it = it_max). */
int vboc_fit_train(vboc_fit_handle h, const vboc_fit_run_t* run, void* stream);

/* `steps` minibatch index draws of the sampler (test hook: the same kernel as the fit; advances the stream) into
 * idx_out (device int32 [steps][minibatch]). */
int vboc_fit_sample(vboc_fit_handle h, long long n, long long n_new, int steps, int* idx_out, void* stream);

int vboc_fit_info(vboc_fit_handle h, int* hidden_padded, int* splits, long long* adam_steps,
                  unsigned long long* draws);
const char* vboc_fit_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
