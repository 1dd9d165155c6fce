// BDPT traversal kernels of one kd stack class (compiled once per class with -DLUMO_STK=<class>,
// see Makefile STK_CLASSES): walk steps, re-runs, (a)-item traces, (b)-item visibility.
#include "launch.h"

#ifndef LUMO_STK
#error "inst_bd.hip is compiled with -DLUMO_STK=<stack class>"
#endif

namespace lumo {
namespace dev {

template <int STK>
void launch_bdpt_step(int grid, hipStream_t sm, int fx, const DScene& sc, const Paths& S, const Tasks& T,
                      const Bdpt& B, const BItems& I, int mode, const int32_t* queue, int32_t* next_queue,
                      uint32_t tail_below) {
    if (fx == 2) k_bdpt_step<STK, 2><<<grid, BLOCK, 0, sm>>>(sc, S, T, B, I, mode, queue, next_queue, tail_below);
    else if (fx) k_bdpt_step<STK, 1><<<grid, BLOCK, 0, sm>>>(sc, S, T, B, I, mode, queue, next_queue, tail_below);
    else k_bdpt_step<STK, 0><<<grid, BLOCK, 0, sm>>>(sc, S, T, B, I, mode, queue, next_queue, tail_below);
}

#define LUMO_TRAV_LAUNCH(KERNEL, ...)                                                        \
    do {                                                                                     \
        if (l.fx == 2) {                                                                     \
            KERNEL<STK, false, 2><<<l.grid, BLOCK, 0, l.sm>>>(__VA_ARGS__);                  \
        } else if (l.lds) {                                                                  \
            if (l.fx) KERNEL<STK, true, true><<<l.grid, BLOCK, l.shm, l.sm>>>(__VA_ARGS__);  \
            else KERNEL<STK, true, false><<<l.grid, BLOCK, l.shm, l.sm>>>(__VA_ARGS__);     \
        } else {                                                                             \
            if (l.fx) KERNEL<STK, false, true><<<l.grid, BLOCK, 0, l.sm>>>(__VA_ARGS__);     \
            else KERNEL<STK, false, false><<<l.grid, BLOCK, 0, l.sm>>>(__VA_ARGS__);        \
        }                                                                                    \
    } while (0)

// ... and, for kernels with a TOP variant (LDS mode 2: scenes too large to stage whole, fx 0 / 1),
// `TB` threads per block with the TOP set (and the kd stack columns) in `l.shm` bytes of LDS.
// The caller asks for TOP (launch_trav's allow_top) only for fx 0 / 1: l.grid is then sized for
// TB-thread blocks, too small a grid for the fallback's BLOCK threads.
// Only the (b)-item visibility has one: TOP variants of the walk (k_closest), the walk tail and
// the (a)-item traces were slower on C4 (the tail 150 -> 239 ms per 8-spp frame, (a) traces
// 177 -> 191 ms), while the visibility went 200 -> 85 ms.
#define LUMO_TRAV_LAUNCH_TOP(KERNEL, TB, ...)                                                 \
    do {                                                                                     \
        if (l.top && l.fx != 2) {                                                            \
            if (l.fx) KERNEL<STK, 2, 1><<<l.grid, TB, l.shm, l.sm>>>(__VA_ARGS__);           \
            else KERNEL<STK, 2, 0><<<l.grid, TB, l.shm, l.sm>>>(__VA_ARGS__);               \
        } else {                                                                             \
            LUMO_TRAV_LAUNCH(KERNEL, __VA_ARGS__);                                           \
        }                                                                                    \
    } while (0)

template <int STK>
void launch_bdpt_tail(const TravLaunch& l, const DScene& sc, const Paths& S, const Tasks& T, const Bdpt& B,
                      const BItems& I, int mode, const int32_t* queue, uint32_t tail_below) {
    LUMO_TRAV_LAUNCH(k_bdpt_tail, sc, S, T, B, I, mode, queue, tail_below);
}

template <int STK>
void launch_bdpt_redo(const TravLaunch& l, const DScene& sc, const Paths& S, const Tasks& T, const DCam& cam,
                      const Bdpt& B, const Bdpt& R, const BItems& I) {
    LUMO_TRAV_LAUNCH(k_bdpt_redo, sc, S, T, cam, B, R, I);
}

template <int STK>
void launch_bdpt_trace_a(const TravLaunch& l, const DScene& sc, const Paths& S, const DCam& cam, const Bdpt& B,
                         const Bdpt& R, const BItems& I, int n, const uint32_t* totals, int kind) {
    LUMO_TRAV_LAUNCH(k_bdpt_trace_a, sc, S, cam, B, R, I, n, totals, kind);
}

template <int STK>
void launch_bdpt_vis(const TravLaunch& l, const DScene& sc, const Paths& S, const Bdpt& B, const Bdpt& R,
                     const BItems& I, int n, uint32_t* totals) {
    LUMO_TRAV_LAUNCH_TOP(k_bdpt_vis, TOP_BLOCK, sc, S, B, R, I, n, totals);
}

template void launch_bdpt_step<LUMO_STK>(int, hipStream_t, int, const DScene&, const Paths&, const Tasks&,
                                         const Bdpt&, const BItems&, int, const int32_t*, int32_t*, uint32_t);
template void launch_bdpt_tail<LUMO_STK>(const TravLaunch&, const DScene&, const Paths&, const Tasks&, const Bdpt&,
                                         const BItems&, int, const int32_t*, uint32_t);
template void launch_bdpt_redo<LUMO_STK>(const TravLaunch&, const DScene&, const Paths&, const Tasks&, const DCam&,
                                         const Bdpt&, const Bdpt&, const BItems&);
template void launch_bdpt_trace_a<LUMO_STK>(const TravLaunch&, const DScene&, const Paths&, const DCam&, const Bdpt&,
                                            const Bdpt&, const BItems&, int, const uint32_t*, int);
template void launch_bdpt_vis<LUMO_STK>(const TravLaunch&, const DScene&, const Paths&, const Bdpt&, const Bdpt&,
                                        const BItems&, int, uint32_t*);

}  // namespace dev
}  // namespace lumo
