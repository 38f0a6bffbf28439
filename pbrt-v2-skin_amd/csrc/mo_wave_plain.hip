// mo_wave_plain.hip -- the sharded gather's wave kernel, spectral, per-band tables (mo_wave.h).
#include "mo_wave.h"

namespace mpss {

void launch_wave_plain(BandArgs a, dim3 grid, bool count, bool wide, bool steal, hipStream_t stream) {
    launch_wave_family<false, false>(a, grid, count, wide, steal, stream);
}

}  // namespace mpss
