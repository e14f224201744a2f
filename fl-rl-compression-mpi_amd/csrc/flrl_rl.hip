// flrl_rl.hip — run-length (RL) encode / decode for MI355X (gfx950).
// (kernels land in the next milestone; entry points report "not implemented")
#include <hip/hip_runtime.h>

#include "flrl.h"
#include "flrl_device.hpp"
#include "flrl_internal.hpp"

using namespace flrl;

extern "C" size_t flrl_rl_scratch_bytes(size_t n) { return 16 + round_up(n / 8 + 16, 16); }
extern "C" size_t flrl_rl_decode_scratch_bytes(size_t runs) { return 16 + round_up(runs / 8 + 16, 16); }

extern "C" int flrl_rl_encode_device(const uint8_t *, size_t, uint8_t *, uint8_t *, uint64_t *,
                                     void *, size_t, void *)
{
    return set_error(FLRL_E_ARG, "flrl_rl_encode_device: not implemented yet");
}

extern "C" int flrl_rl_decode_device(const uint8_t *, const uint8_t *, size_t, uint8_t *, size_t,
                                     void *, size_t, void *)
{
    return set_error(FLRL_E_ARG, "flrl_rl_decode_device: not implemented yet");
}

extern "C" int flrl_rl_compress(const uint8_t *, size_t, flrl_rl_buf *)
{
    return set_error(FLRL_E_ARG, "flrl_rl_compress: not implemented yet");
}

extern "C" int flrl_rl_decompress(size_t, const uint8_t *, const uint8_t *, size_t, uint8_t **,
                                  size_t *)
{
    return set_error(FLRL_E_ARG, "flrl_rl_decompress: not implemented yet");
}
