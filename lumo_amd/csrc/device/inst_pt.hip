// Path-tracing traversal kernels of one kd stack class (compiled once per class with
// -DLUMO_STK=<class>, see Makefile STK_CLASSES): k_closest, k_shadow, k_trace and their launchers.
#include <cstdio>
#include <cstdlib>

#include "launch.h"
#include "pt.h"

#ifndef LUMO_STK
#error "inst_pt.hip is compiled with -DLUMO_STK=<stack class>"
#endif

namespace lumo {
namespace dev {

template <int STK>
void launch_closest(const TravLaunch& l, const DScene& sc, const Paths& S, const int32_t* queue, uint32_t tail_below) {
    if (l.lds) {
        if (l.fx) k_closest<STK, true, true><<<l.grid, BLOCK, l.shm, l.sm>>>(sc, S, queue, tail_below);
        else k_closest<STK, true, false><<<l.grid, BLOCK, l.shm, l.sm>>>(sc, S, queue, tail_below);
    } else {
        if (l.fx) k_closest<STK, false, true><<<l.grid, BLOCK, 0, l.sm>>>(sc, S, queue, tail_below);
        else k_closest<STK, false, false><<<l.grid, BLOCK, 0, l.sm>>>(sc, S, queue, tail_below);
    }
}

template <int STK>
void launch_closest_q(const TravLaunch& l, const DScene& sc, const Paths& S, const QState& cur, uint32_t skip_below) {
    if (l.top) {
        if (l.fx) k_closest_q<STK, 2, true><<<l.grid, TOP_BLOCK, l.shm, l.sm>>>(sc, S, cur, skip_below);
        else k_closest_q<STK, 2, false><<<l.grid, TOP_BLOCK, l.shm, l.sm>>>(sc, S, cur, skip_below);
    } else if (l.lds) {
        if (l.fx) k_closest_q<STK, true, true><<<l.grid, BLOCK, l.shm, l.sm>>>(sc, S, cur, skip_below);
        else k_closest_q<STK, true, false><<<l.grid, BLOCK, l.shm, l.sm>>>(sc, S, cur, skip_below);
    } else {
        if (l.fx) k_closest_q<STK, false, true><<<l.grid, BLOCK, 0, l.sm>>>(sc, S, cur, skip_below);
        else k_closest_q<STK, false, false><<<l.grid, BLOCK, 0, l.sm>>>(sc, S, cur, skip_below);
    }
}

template <int STK, bool NS1>
void launch_shadow_q_ns(const TravLaunch& l, const DScene& sc, const Paths& S, const QState& nxt) {
    if (l.top) {  // TOP staging: the BVHs' top levels and the object records in LDS
        if (l.fx == 2) k_shadow_q<STK, 2, 2, NS1><<<l.grid, TOP_BLOCK, l.shm, l.sm>>>(sc, S, nxt);
        else if (l.fx) k_shadow_q<STK, 2, 1, NS1><<<l.grid, TOP_BLOCK, l.shm, l.sm>>>(sc, S, nxt);
        else k_shadow_q<STK, 2, 0, NS1><<<l.grid, TOP_BLOCK, l.shm, l.sm>>>(sc, S, nxt);
    } else if (l.fx == 2) {  // textured scenes: emission textures (no whole-scene LDS staging variant)
        k_shadow_q<STK, false, 2, NS1><<<l.grid, BLOCK, 0, l.sm>>>(sc, S, nxt);
    } else if (l.lds) {
        if (l.fx) k_shadow_q<STK, true, true, NS1><<<l.grid, BLOCK, l.shm, l.sm>>>(sc, S, nxt);
        else k_shadow_q<STK, true, false, NS1><<<l.grid, BLOCK, l.shm, l.sm>>>(sc, S, nxt);
    } else {
        if (l.fx) k_shadow_q<STK, false, true, NS1><<<l.grid, BLOCK, 0, l.sm>>>(sc, S, nxt);
        else k_shadow_q<STK, false, false, NS1><<<l.grid, BLOCK, 0, l.sm>>>(sc, S, nxt);
    }
}

template <int STK>
void launch_shadow_q(const TravLaunch& l, const DScene& sc, const Paths& S, const QState& nxt) {
    if (sc.n_shadow == 1)
        launch_shadow_q_ns<STK, true>(l, sc, S, nxt);
    else
        launch_shadow_q_ns<STK, false>(l, sc, S, nxt);
}

template <int STK>
void launch_bounce_q(const TravLaunch& l, const DScene& sc, const Paths& S, const Tasks& T, const QState& cur,
                     const QState& nxt, uint32_t tail_below, bool tail_only, int dyn, int threads) {
    // fused bounce: `threads` per block (64 / 128 / 256), 12 doubles of LDS per thread for the
    // B record after the staged scene; the tail kernel keeps BLOCK threads and needs no record LDS
    const int nt = tail_only ? BLOCK : threads;
    const int grid = l.grid * (BLOCK / nt);
    const size_t rec = tail_only ? 0 : (size_t)PARK_DOUBLES * sizeof(double) * nt;
    const size_t scene = l.lds ? (l.shm + 15) / 16 * 16 : 0;
#if LUMO_BOUNCE_ARGPTR
    if (!l.args) {  // every stream of a context has its block (launch_trav)
        std::fprintf(stderr, "lumo_amd: k_bounce_q launched on a stream without an argument block\n");
        std::abort();
    }
    k_put_args<STK><<<1, 64, 0, l.sm>>>(BounceArgs{sc, S, T, cur, nxt}, l.args);
#define LUMO_BQ_ARGS (l.args, tail_below, dyn)
#else
#define LUMO_BQ_ARGS (sc, S, T, cur, nxt, tail_below, dyn)
#endif
    auto go = [&](auto TL) {
        constexpr bool TAIL = decltype(TL)::value;
        if (l.fx == 2) {  // textured scenes: no LDS staging variant (as k_shadow_q)
            k_bounce_q<STK, false, 2, TAIL><<<grid, nt, rec, l.sm>>>LUMO_BQ_ARGS;
        } else if (l.lds) {
            if (l.fx)
                k_bounce_q<STK, true, 1, TAIL><<<grid, nt, scene + rec, l.sm>>>LUMO_BQ_ARGS;
            else
                k_bounce_q<STK, true, 0, TAIL><<<grid, nt, scene + rec, l.sm>>>LUMO_BQ_ARGS;
        } else {
            if (l.fx) k_bounce_q<STK, false, 1, TAIL><<<grid, nt, rec, l.sm>>>LUMO_BQ_ARGS;
            else k_bounce_q<STK, false, 0, TAIL><<<grid, nt, rec, l.sm>>>LUMO_BQ_ARGS;
        }
    };
    if (tail_only)
        go(std::true_type{});
    else
        go(std::false_type{});
#undef LUMO_BQ_ARGS
}

template <int STK>
void launch_trace(int grid, hipStream_t sm, const DScene& sc, const double* o, const double* d, const int32_t* light,
                  int n, int any_hit, double* t_out, int32_t* kind_out, int32_t* obj_out, int32_t* prim_out,
                  unsigned long long* tcount, bool top) {
    if (top)
        k_trace<STK, true><<<grid, TOP_BLOCK, sc.top_shm, sm>>>(sc, o, d, light, n, any_hit, t_out, kind_out, obj_out,
                                                                  prim_out, tcount);
    else
        k_trace<STK, false><<<grid, BLOCK, 0, sm>>>(sc, o, d, light, n, any_hit, t_out, kind_out, obj_out, prim_out,
                                                    tcount);
}

template void launch_closest<LUMO_STK>(const TravLaunch&, const DScene&, const Paths&, const int32_t*, uint32_t);
template void launch_closest_q<LUMO_STK>(const TravLaunch&, const DScene&, const Paths&, const QState&, uint32_t);
template void launch_shadow_q<LUMO_STK>(const TravLaunch&, const DScene&, const Paths&, const QState&);
template void launch_bounce_q<LUMO_STK>(const TravLaunch&, const DScene&, const Paths&, const Tasks&, const QState&,
                                        const QState&, uint32_t, bool, int, int);
template void launch_trace<LUMO_STK>(int, hipStream_t, const DScene&, const double*, const double*, const int32_t*,
                                     int, int, double*, int32_t*, int32_t*, int32_t*, unsigned long long*, bool);

}  // namespace dev
}  // namespace lumo
