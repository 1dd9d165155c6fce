// Launchers of the traversal kernels, one explicit instantiation per kd stack class STK.  Each
// class is compiled in its own translation units (inst_pt.hip / inst_bd.hip built with
// -DLUMO_STK=<class>), so the kernel instantiations build in parallel; kernels.hip only calls
// these functions.
#pragma once
#include "bdpt.h"

namespace lumo {
namespace dev {

// kd stack classes the kernels are instantiated for (Makefile STK_CLASSES must match; it also
// builds class 0, the wide accel's walks, dscene.h wide_walk).
constexpr int STACK_CLASSES[] = {4, 8, 16, 24, 32, 48, 64};

// Launch geometry of a traversal kernel: grid, dynamic LDS (staged scene), LDS staging on/off,
// feature class (FX), stream.
struct TravLaunch {
    int grid;
    size_t shm;
    bool lds;
    int fx;  // feature class (dscene.h): 0 lean, 1 full, 2 full + textures
    hipStream_t sm;
    // TOP staging (k_closest_q / k_shadow_q of scenes too large for `lds`): TOP_BLOCK threads per
    // block, `shm` bytes of LDS (DScene::top_bytes), grid `grid`
    bool top = false;
    BounceArgs* args = nullptr;  // this stream's BounceArgs block (k_bounce_q, LUMO_BOUNCE_ARGPTR)
};

template <int STK>
void launch_closest(const TravLaunch& l, const DScene& sc, const Paths& S, const int32_t* queue, uint32_t tail_below);
template <int STK>
void launch_closest_q(const TravLaunch& l, const DScene& sc, const Paths& S, const QState& cur, uint32_t skip_below);
template <int STK>
void launch_shadow_q(const TravLaunch& l, const DScene& sc, const Paths& S, const QState& nxt);
template <int STK>
void launch_bounce_q(const TravLaunch& l, const DScene& sc, const Paths& S, const Tasks& T, const QState& cur,
                     const QState& nxt, uint32_t tail_below, bool tail_only, int dyn, int threads);
template <int STK>
void launch_trace(int grid, hipStream_t sm, const DScene& sc, const double* o, const double* d, const int32_t* light,
                  int n, int any_hit, double* t_out, int32_t* kind_out, int32_t* obj_out, int32_t* prim_out,
                  unsigned long long* tcount, bool top);

template <int STK>
void launch_bdpt_step(int grid, hipStream_t sm, int fx, const DScene& sc, const Paths& S, const Tasks& T,
                      const Bdpt& B, const BItems& I, int mode, const int32_t* queue, int32_t* next_queue,
                      uint32_t tail_below);
template <int STK>
void launch_bdpt_tail(const TravLaunch& l, const DScene& sc, const Paths& S, const Tasks& T, const Bdpt& B,
                      const BItems& I, int mode, const int32_t* queue, uint32_t tail_below);
template <int STK>
void launch_bdpt_redo(const TravLaunch& l, const DScene& sc, const Paths& S, const Tasks& T, const DCam& cam,
                      const Bdpt& B, const Bdpt& R, const BItems& I);
template <int STK>
void launch_bdpt_trace_a(const TravLaunch& l, const DScene& sc, const Paths& S, const DCam& cam, const Bdpt& B,
                         const Bdpt& R, const BItems& I, int n, const uint32_t* totals, int kind);
template <int STK>
void launch_bdpt_vis(const TravLaunch& l, const DScene& sc, const Paths& S, const Bdpt& B, const Bdpt& R,
                     const BItems& I, int n, uint32_t* totals);

#define LUMO_EXTERN_STK(K)                                                                                        \
    extern template void launch_closest<K>(const TravLaunch&, const DScene&, const Paths&, const int32_t*,        \
                                           uint32_t);                                                             \
    extern template void launch_closest_q<K>(const TravLaunch&, const DScene&, const Paths&, const QState&,       \
                                             uint32_t);                                                           \
    extern template void launch_shadow_q<K>(const TravLaunch&, const DScene&, const Paths&, const QState&);        \
    extern template void launch_bounce_q<K>(const TravLaunch&, const DScene&, const Paths&, const Tasks&,        \
                                            const QState&, const QState&, uint32_t, bool, int, int);             \
    extern template void launch_trace<K>(int, hipStream_t, const DScene&, const double*, const double*,          \
                                         const int32_t*, int, int, double*, int32_t*, int32_t*, int32_t*,         \
                                         unsigned long long*, bool);                                              \
    extern template void launch_bdpt_step<K>(int, hipStream_t, int, const DScene&, const Paths&, const Tasks&,   \
                                             const Bdpt&, const BItems&, int, const int32_t*, int32_t*,           \
                                             uint32_t);                                                           \
    extern template void launch_bdpt_tail<K>(const TravLaunch&, const DScene&, const Paths&, const Tasks&,        \
                                             const Bdpt&, const BItems&, int, const int32_t*, uint32_t);          \
    extern template void launch_bdpt_redo<K>(const TravLaunch&, const DScene&, const Paths&, const Tasks&,        \
                                             const DCam&, const Bdpt&, const Bdpt&, const BItems&);               \
    extern template void launch_bdpt_trace_a<K>(const TravLaunch&, const DScene&, const Paths&, const DCam&,      \
                                                const Bdpt&, const Bdpt&, const BItems&, int, const uint32_t*,    \
                                                int);                                                             \
    extern template void launch_bdpt_vis<K>(const TravLaunch&, const DScene&, const Paths&, const Bdpt&,          \
                                            const Bdpt&, const BItems&, int, uint32_t*);
#ifndef LUMO_STK
LUMO_EXTERN_STK(0)
LUMO_EXTERN_STK(4)
LUMO_EXTERN_STK(8)
LUMO_EXTERN_STK(16)
LUMO_EXTERN_STK(24)
LUMO_EXTERN_STK(32)
LUMO_EXTERN_STK(48)
LUMO_EXTERN_STK(64)
#endif

}  // namespace dev
}  // namespace lumo
