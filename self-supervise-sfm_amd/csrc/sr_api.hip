// Host-side ABI plumbing: error reporting, version, the last launched kernel's name, the tuning
// switches (sfm_amd.h sr_tuning_key) and the SR_TUNE_SYNC_CHECK debug mode.
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <mutex>

#include "sr_common.h"

namespace {
thread_local char g_err[512] = "";
thread_local char g_kernel[128] = "";

struct TuneDef {
  const char* env;
  int def;
};
// index = sr_tuning_key
constexpr TuneDef kTune[SR_TUNE_COUNT] = {
    {"SR_ATTN_MZERO", 1}, {"SR_ATTN_CFG", -1}, {"SR_ATTN_PIPE", 1}, {"SR_ATTN_PIPE_SEG", 0},
    {"SR_ATTN_NO_SHORT", 0}, {"SR_GEMM_GROUP_M", -1}, {"SR_GEMM_SMALLM", 1}, {"SR_GEMM_NO256", 0},
    {"SR_GEMM_REG_EPI", 0}, {"SR_CONV_NO_NARROW", 0}, {"SR_WGRAD256", 1}, {"SR_SYNC_CHECK", 0},
    {"SR_RLN_WIDE", 0}, {"SR_GEMM_TAIL", 1}, {"SR_GEMM_RESID_LDS", 1}, {"SR_GEMM_ROPE_LDS", 1},
    {"SR_ATTN_BWD_PIPE", 1}, {"SR_ATTN_BWD_DQ_PIPE", 1}, {"SR_ATTN_BWD_CAT", 1},
};
std::atomic<int> g_tune[SR_TUNE_COUNT];
std::once_flag g_tune_once;

void tune_init() {
  std::call_once(g_tune_once, [] {
    for (int k = 0; k < SR_TUNE_COUNT; ++k) {
      const char* e = getenv(kTune[k].env);
      // a set-but-empty variable (the old "defined = on" switches) reads as 1
      g_tune[k].store(e ? (*e ? atoi(e) : 1) : kTune[k].def, std::memory_order_relaxed);
    }
  });
}
}  // namespace

namespace sr {

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

void note_kernel(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_kernel, sizeof(g_kernel), fmt, ap);
  va_end(ap);
}

int tune(int key) {
  tune_init();
  return g_tune[key].load(std::memory_order_relaxed);
}

int cu_count() {
  static std::once_flag once;
  static int n = 256;
  std::call_once(once, [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      n = v;
  });
  return n;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e == hipSuccess && tune(SR_TUNE_SYNC_CHECK)) {
    // debug mode: attribute an asynchronous fault to the call that launched it
    e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipGetLastError();
    if (e != hipSuccess) {
      set_error("%s: kernel %s failed (SR_SYNC_CHECK): %s", what, g_kernel, hipGetErrorString(e));
      return SR_ELAUNCH;
    }
  }
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return SR_ELAUNCH;
  }
  return SR_OK;
}

}  // namespace sr

extern "C" const char* sr_last_error(void) { return g_err; }
extern "C" const char* sr_last_kernel(void) { return g_kernel; }
extern "C" int sr_version(void) { return (1 << 16) | 5; }  // 1.1: sr_gemm_wgrad_pair; 1.2: sr_attention_bwd_f32; 1.3: tuning keys renumbered; 1.4: sr_gemm_epi.colsum; 1.5: sr_attention_pair_vt, sr_vt_tiles, sr_colsum_fma, sr_vec_fma2_f32

extern "C" int sr_set_tuning(int key, int value) {
  SR_CHECK(key >= 0 && key < SR_TUNE_COUNT, SR_EINVAL, "sr_set_tuning: unknown key %d", key);
  tune_init();
  return g_tune[key].exchange(value, std::memory_order_relaxed);
}

extern "C" int sr_get_tuning(int key) {
  SR_CHECK(key >= 0 && key < SR_TUNE_COUNT, SR_EINVAL, "sr_get_tuning: unknown key %d", key);
  return sr::tune(key);
}

extern "C" const char* sr_tuning_name(int key) {
  return key >= 0 && key < SR_TUNE_COUNT ? kTune[key].env : nullptr;
}
