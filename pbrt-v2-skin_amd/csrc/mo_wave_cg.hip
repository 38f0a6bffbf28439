// mo_wave_cg.hip -- the sharded gather's wave kernel, spectral, common grid (mo_wave.h).
#include "mo_wave.h"

namespace mpss {

void launch_wave_cg(BandArgs a, dim3 grid, bool count, bool wide, bool steal, hipStream_t stream) {
    launch_wave_family<true, false>(a, grid, count, wide, steal, stream);
}

}  // namespace mpss
