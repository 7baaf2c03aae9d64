// Device-side checks of the debug build (QFEDX_DEBUG=1 -> extension _qfedx_C_debug, -DQFX_DEVICE_CHECKS=1).
//
// A failed QFX_DCHECK records the first failing source line in a per-translation-unit device status word and
// the kernel carries on: no trap (a trapping or faulting kernel can reset every GPU of a shared node), LDS
// accesses past the allocation are dropped by the hardware, and every global extent is validated on the host
// before launch.  The bindings read and clear the word after each launch of the debug build and raise with
// the line.  In the release build the checks compile to nothing.
#pragma once

#if defined(QFX_DEVICE_CHECKS) && QFX_DEVICE_CHECKS
#define QFX_CHECKS_ON 1
#define QFX_DCHECK(cond)                                                       \
  do {                                                                         \
    if (!(cond)) atomicCAS(&qfx_check_word, 0u, (unsigned int)__LINE__);       \
  } while (0)
#else
#define QFX_CHECKS_ON 0
#define QFX_DCHECK(cond) ((void)0)
#endif
