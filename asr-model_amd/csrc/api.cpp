// C-ABI plumbing: thread-local last-error string and launch checking.
#include "common.h"

namespace asrx {

static thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return (int)e;
  }
  return 0;
}

}  // namespace asrx

extern "C" {

const char* asrx_last_error(void) { return asrx::g_last_error.c_str(); }

int asrx_abi_version(void) { return 1; }

int asrx_set_noise_epoch_abby(uint32_t epoch, hipStream_t stream);
int asrx_set_noise_epoch_rowops(uint32_t epoch, hipStream_t stream);

// Noise epoch of every noise-drawing kernel (see common.h): stream-ordered, so a graph replayed on
// `stream` after this call draws the epoch's noise.  0 = the oracle's keys.
int asrx_set_noise_epoch(uint32_t epoch, hipStream_t stream) {
  int e = asrx_set_noise_epoch_abby(epoch, stream);
  return e ? e : asrx_set_noise_epoch_rowops(epoch, stream);
}

// Host-side restatement of the device noise hash (used by tests to cross-check oracle/noise.py).
uint32_t asrx_noise_hash(uint32_t key, uint32_t idx) {
  return asrx::mix32(asrx::mix32(idx ^ key) + (key * 0x9E3779B9U + 0x632BE5ABU));
}

}
