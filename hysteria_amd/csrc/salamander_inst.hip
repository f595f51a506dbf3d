// salamander_inst.hip -- instantiates the batch kernels for one salt word
// (compiled once per HY_SW = 0..15, see Makefile).
#include "salamander_flat.h"

#ifndef HY_SW
#error "compile with -DHY_SW=<salt word 0..15>"
#endif

namespace hyobfs {
template void launch_wave_sw<true, true, HY_SW>(const BatchParams&, const KeyParams&, hipStream_t);
template void launch_wave_sw<true, false, HY_SW>(const BatchParams&, const KeyParams&, hipStream_t);
template void launch_wave_sw<false, true, HY_SW>(const BatchParams&, const KeyParams&, hipStream_t);
template void launch_wave_sw<false, false, HY_SW>(const BatchParams&, const KeyParams&, hipStream_t);
template void launch_tile_sw<true, HY_SW>(const BatchParams&, const KeyParams&, const TileParams&, hipStream_t);
template void launch_tile_sw<false, HY_SW>(const BatchParams&, const KeyParams&, const TileParams&, hipStream_t);
template void launch_flat_sw<true, HY_SW>(const BatchParams&, const KeyParams&, const FlatParams&, hipStream_t);
template void launch_flat_sw<false, HY_SW>(const BatchParams&, const KeyParams&, const FlatParams&, hipStream_t);
}  // namespace hyobfs
