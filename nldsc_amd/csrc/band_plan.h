// band_plan.h — host-side window replay (ChunkwiseReader, stream.h:131-155,182-197) and the band kernel's
// work-item schedule; host-only C++ (no HIP), shared by ld_engine.cpp and the sanitizer build.
#pragma once
#include <cstdint>
#include <vector>

namespace nldsc {

// one work item of the band kernels: row block x, first column block y, z column blocks (1 or 2), w = 0;
// uploaded as the kernels' int4 (same 16-byte layout)
struct PlanItem {
    int32_t x, y, z, w;
};
static_assert(sizeof(PlanItem) == 16, "PlanItem is the device int4");

void replay_windows(const double* pos, const uint8_t* flags, int n, double w, int* L, int* R);
bool positions_sorted(const double* pos, int M);
bool positions_nonneg_sorted(const double* pos, int M);
void plan_items(const double* pos, const uint8_t* flags, int M, double w, const int* L, const int* R, int own_begin,
                int own_end, int max_nc, std::vector<PlanItem>& out);
void order_items_tiled(std::vector<PlanItem>& items, int nblk, int R, int C, std::vector<PlanItem>& scratch);

}  // namespace nldsc
