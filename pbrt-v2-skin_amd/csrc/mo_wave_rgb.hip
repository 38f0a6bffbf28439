// mo_wave_rgb.hip -- the sharded gather's wave kernel, rgbprofile, per-band tables (mo_wave.h).
#include "mo_wave.h"

namespace mpss {

void launch_wave_rgb(BandArgs a, dim3 grid, bool count, bool wide, bool steal, hipStream_t stream) {
    launch_wave_family<false, true>(a, grid, count, wide, steal, stream);
}

}  // namespace mpss
