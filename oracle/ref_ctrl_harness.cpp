/*
 * ref_ctrl_harness.cpp -- driver around the REFERENCE's own motor speed controller
 * UTIL::FF_PI_D (src/Utility/util_controller.hpp:155-186, with UTIL::PI_D :92-153 and
 * the UTIL::IIR1 velocity low-pass of src/Utility/util_iir.hpp:13-57), compiled
 * unmodified from /root/reference by oracle/Makefile into oracle/_ref/libctrl_ref.so.
 *
 * TEST INFRASTRUCTURE ONLY.  util_controller.hpp includes nothing but util_iir.hpp, so
 * no stand-in of any kind is involved.  The harness constructs the controller the way
 * VD_task_main.cpp:86-89,157-160 does (or with the caller's gains) and replays a
 * sequence of set_target / update / reset calls, recording what the reference returns,
 * so tests/golden/ can pin the oracle's restatement (oracle/fmskf_oracle.c orc_pid_*).
 * Built with -ffp-contract=off like the oracle: the source semantics, no contraction.
 */
#include <stdint.h>

#include "util_controller.hpp"

extern "C" {

/* Replay n steps on one FF_PI_D.  Step k: if reset[k] -> reset(); set_target(tgt[k]);
 * ctrl[k] = update(val[k]); now_val[k] = get_now_val(); target[k] = get_target(). */
int ref_ffpid_run(float c_freq, float ff_gain, float p_gain, float i_gain, float d_gain,
                  float i_limit, float lpf_freq, float ff_limit, int n, const float *tgt,
                  const float *val, const uint8_t *reset, float *ctrl, float *now_val,
                  float *target) {
  UTIL::FF_PI_D c(c_freq, ff_gain, p_gain, i_gain, d_gain, i_limit, lpf_freq);
  c.set_FF_limit(ff_limit);
  for (int k = 0; k < n; k++) {
    if (reset && reset[k]) c.reset();
    c.set_target(tgt[k]);
    ctrl[k] = c.update(val[k]);
    now_val[k] = c.get_now_val();
    target[k] = c.get_target();
  }
  return 0;
}

/* UTIL::IIR1 alone: y[k] = update(x[k]) */
int ref_iir1_run(float a1, float b0, float b1, int n, const float *x, float *y) {
  UTIL::IIR1 f(a1, b0, b1);
  for (int k = 0; k < n; k++) y[k] = f.update(x[k]);
  return 0;
}

}  // extern "C"
