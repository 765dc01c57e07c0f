// engine.cpp — the rank-local protocol loops of the partitioned solves: the
// MI355X form of the reference's bulk-synchronous round loop
// (ParallelJohnson.cpp:488-594). Every rank runs the same loop; the only
// cross-rank traffic is the Comm calls, made in the same order on every rank.
//
// BFS (unit weights, the reference's w = 1, :147): one level per round. A level
// is a push (the owned frontier expands; ids owned elsewhere are sent to their
// owner, the Alltoall + Alltoallv of :522-554) or a pull (owned unvisited
// vertices probe their in-neighbours in a replicated visited bitmap that is
// all-gathered around pull levels). Beamer's rule on all-reduced counts picks
// the direction, identically on every rank; a zero global frontier ends the
// solve (the termination Allreduce of :579-593).
//
// Delta-stepping (weighted): bands [lo, lo + delta) in order; light rounds
// until no rank has a frontier, then one heavy step; candidates for remote
// vertices are exchanged as (id | dist << 32). An empty band jumps to the band
// of the all-reduced minimum pending distance; INT_INF everywhere ends it.
#include <chrono>
#include <cstring>

#include "engine.h"

namespace pj {

namespace {

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// When a rank fails mid-protocol, its peers would wait forever at the next
// collective: release them (thread groups) before rethrowing.
template <typename F>
void guarded_loop(Comm& comm, F&& f) {
    try {
        f();
    } catch (...) {
        comm.abort();
        throw;
    }
}

}  // namespace

// A transport other than "self" exchanges even at world 1 (nothing is sent
// then), so a one-GPU run exercises the same collective calls as a group.
static bool exchanges(const Comm& comm) { return comm.world > 1 || std::strcmp(comm.kind(), "self") != 0; }

void bfs_engine(BfsSteps& S, Comm& comm, i64 source, const BfsParams& prm, bool iso_ready, pj_part_stats* st) {
    if (comm.world != S.world || comm.rank != S.rank)
        throw Error(PJ_ERR_COMM, "transport rank/world differ from the partition's");
    guarded_loop(comm, [&] {
        hipStream_t s = S.stream();
        const double t0 = now_ms();
        const size_t slice = (size_t)S.bw * sizeof(u64);
        if (!iso_ready) {  // replicated isolated-vertex mask: one all-gather per graph and transport
            S.zmask();
            comm.allgather(S.zown, S.iso, slice, s);
        }
        i64 nnz_global = S.nnz_local;
        comm.allreduce(&nnz_global, 1, false, s);
        auto gather_vis = [&] {
            if (exchanges(comm))
                comm.allgather(static_cast<char*>(S.vis) + (size_t)S.rank * slice, S.vis, slice, s);
        };
        i64 f[3];
        S.begin(source, f);
        comm.allreduce(f, 3, false, s);
        // device rows (RCCL): a level's counts exchange and its termination statistics
        // each cost one collective and one host wait, with no readback by the step
        const bool dev = comm.rows_on_device() && S.counts_dev() && S.stats_dev();
        std::vector<i64> rows((size_t)S.world * (size_t)std::max(S.world, 5));
        auto end_level = [&](i64* f3) {
            if (!dev) {
                S.end_level(f3);
                comm.allreduce(f3, 3, false, s);
                return;
            }
            S.end_level_async();
            comm.allgather_rows_dev(S.stats_dev(), 5, rows.data(), s);
            // a foreign id received by any rank fails every rank at the same level (a peer
            // of a multi-process group would otherwise wait in the next collective)
            for (int q = 0; q < S.world; ++q)
                if (q != S.rank && rows[5 * (size_t)q + 4])
                    throw Error(PJ_ERR_COMM, "rank " + std::to_string(q) +
                                                 " received ids owned by another rank (corrupted exchange)");
            S.end_level_finish(rows.data() + 5 * (size_t)S.rank);
            f3[0] = f3[1] = f3[2] = 0;
            for (int q = 0; q < S.world; ++q)
                for (int j = 0; j < 3; ++j) f3[j] += rows[5 * (size_t)q + (size_t)j];
        };
        i64 n_f = f[0], m_f = f[1];
        i64 n_r = n_f, m_r = m_f, m_u = nnz_global - m_f;
        int mode = 0, level = 0;
        i64 td = 0, bu = 0, sent = 0;
        if (prm.force == 2) {
            mode = 1;
            gather_vis();
        }
        std::vector<i64> counts((size_t)S.world), rcounts((size_t)S.world);
        while (n_f > 0 && level + 1 < INT_INF) {
            const i64 prev_n_f = n_f;
            if (mode == 0) {
                i64 nr = 0;
                if (dev) {
                    S.push(level, nullptr);
                    comm.allgather_rows_dev(S.counts_dev(), S.world, rows.data(), s);
                    for (int q = 0; q < S.world; ++q) {
                        counts[(size_t)q] = rows[(size_t)S.rank * S.world + (size_t)q];
                        rcounts[(size_t)q] = rows[(size_t)q * S.world + (size_t)S.rank];
                    }
                } else {
                    S.push(level, counts.data());
                    if (exchanges(comm)) comm.alltoall_counts(counts.data(), rcounts.data(), s);
                }
                i64 npieces = 1;
                if (exchanges(comm)) {
                    i64 ns = 0;
                    for (int q = 0; q < S.world; ++q) {
                        ns += q == S.rank ? 0 : counts[(size_t)q];
                        nr += rcounts[(size_t)q];
                    }
                    const i64 cap = S.exchange_cap();
                    if (cap > 0) {  // the pieces every rank uses: from the largest side of any rank
                        i64 need = -std::max(ns, nr);  // (max over ranks as a min of negatives)
                        comm.allreduce(&need, 1, true, s);
                        need = -need;
                        // pieces of about cap / 2 (a piece of a skewed level may exceed its share)
                        const i64 half = std::max<i64>(1, cap / 2);
                        if (need > cap) npieces = std::min<i64>((need + half - 1) / half, std::max<i64>(1, S.bw));
                    }
                    if (npieces <= 1) {
                        S.exchange_buffers(ns, nr);
                        comm.alltoallv(S.send, counts.data(), S.recv, rcounts.data(), sizeof(u32), s);
                        sent += ns;
                    }
                }
                if (npieces <= 1) {
                    S.apply(level, nr);
                } else {
                    for (int k = 0; k < (int)npieces; ++k) {
                        S.piece_counts(k, (int)npieces, counts.data());
                        comm.alltoall_counts(counts.data(), rcounts.data(), s);
                        i64 ns = 0, nrk = 0;
                        for (int q = 0; q < S.world; ++q) {
                            ns += q == S.rank ? 0 : counts[(size_t)q];
                            nrk += rcounts[(size_t)q];
                        }
                        S.exchange_buffers(ns, nrk);
                        comm.alltoallv(S.send, counts.data(), S.recv, rcounts.data(), sizeof(u32), s);
                        sent += ns;
                        S.apply(level, nrk);
                    }
                }
                ++td;
            } else {
                S.pull(level);
                ++bu;
            }
            end_level(f);
            n_f = f[0];
            m_f = f[1];
            n_r += n_f;
            m_r += m_f;
            m_u -= m_f;
            // Beamer: pull when the frontier's edges exceed the unexplored edges / alpha,
            // back to push when the frontier is small and shrinking
            int nxt = mode;
            if (prm.force == 1) nxt = 0;
            else if (prm.force == 2) nxt = 1;
            else if (mode == 0 && (double)m_f > (double)m_u / prm.alpha) nxt = 1;
            else if (mode == 1 && (double)n_f < (double)S.n / prm.beta && n_f < prev_n_f) nxt = 0;
            if (n_f > 0 && (nxt == 1 || mode == 1)) gather_vis();
            mode = nxt;
            ++level;
        }
        comm.sync(s);
        if (st) {
            *st = pj_part_stats{};
            st->solve_ms = now_ms() - t0;
            st->levels = level;
            st->td_levels = td;
            st->bu_levels = bu;
            st->reached = n_r;
            st->reached_edges = m_r;
            st->sent = sent;
        }
    });
}

void delta_engine(DeltaSteps& S, Comm& comm, i64 source, int32_t delta_in, pj_part_stats* st) {
    if (comm.world != S.world || comm.rank != S.rank)
        throw Error(PJ_ERR_COMM, "transport rank/world differ from the partition's");
    guarded_loop(comm, [&] {
        hipStream_t s = S.stream();
        const double t0 = now_ms();
        int32_t delta = S.begin(source, delta_in);
        const int32_t delta0 = delta;
        // tail switch: every rank takes the same decision from the all-reduced counts
        const double tfrac = S.tail_frac();
        const int32_t tdelta = S.tail_delta(delta);
        i64 all_edges = 0;
        bool tail_on = tfrac > 0.0 && tdelta > delta;
        if (tail_on) {
            all_edges = S.local_edges();
            comm.allreduce(&all_edges, 1, false, s);
        }
        // the pull rules: agreed once per solve (any rank vetoes: a rank whose rows are not
        // its in-edges, or with a pull off), so a vetoed pull costs no per-band collective
        const double pf = S.pull_factor(), lpf0 = S.light_pull_factor(), tlpf = S.tail_light_pull_factor();
        i64 allow[3] = {pf > 0.0 ? 1 : 0, lpf0 > 0.0 ? 1 : 0, tlpf > 0.0 ? 1 : 0};
        comm.allreduce(allow, 3, false, s);
        const bool heavy_pull_ok = allow[0] == S.world, tail_light_ok = allow[2] == S.world;
        bool light_pull_ok = allow[1] == S.world;
        double lpf = lpf0;
        const i64 map_w = S.pull_map_width();
        std::vector<i64> counts((size_t)S.world), rcounts((size_t)S.world);
        i64 sent = 0, bands = 0, rounds = 0, pulls = 0, lpulls = 0;
        auto exchange_apply = [&](int light, int32_t lo, int32_t hi) {
            S.relax(light, lo, hi, counts.data());
            i64 nr = 0;
            if (exchanges(comm)) {
                comm.alltoall_counts(counts.data(), rcounts.data(), s);
                i64 ns = 0;
                for (int q = 0; q < S.world; ++q) {
                    ns += counts[(size_t)q];
                    nr += rcounts[(size_t)q];
                }
                S.exchange_buffers(ns, nr);
                comm.alltoallv(S.send, counts.data(), S.recv, rcounts.data(), sizeof(u64), s);
                sent += ns;
            }
            S.apply(nr, light, lo, hi);
        };
        // device rows (RCCL): a band's size and min pending distance in one collective, a
        // round's frontier size in one, each with one host wait
        const bool dev = comm.rows_on_device() && S.select_dev() && S.nf_dev();
        std::vector<i64> rows((size_t)S.world * 2);
        i64 lo = 0;
        while (lo < INT_INF) {
            const i64 hi = std::min<i64>(lo + delta, INT_INF);
            i64 cnt = 0, mn = INT_INF;
            if (dev) {
                S.select_async((int32_t)lo, (int32_t)hi);
                comm.allgather_rows_dev(S.select_dev(), 2, rows.data(), s);
                S.select_finish();
                for (int q = 0; q < S.world; ++q) {
                    const u64 m = (u64)rows[2 * (size_t)q];
                    mn = std::min<i64>(mn, m >= (u64)INT_INF ? (i64)INT_INF : (i64)m);
                    cnt += rows[2 * (size_t)q + 1];
                }
            } else {
                i64 sel[2];
                S.select((int32_t)lo, (int32_t)hi, sel);
                cnt = sel[0];
                comm.allreduce(&cnt, 1, false, s);
                if (cnt == 0) {
                    mn = sel[1];
                    comm.allreduce(&mn, 1, true, s);
                }
            }
            if (cnt == 0) {
                if (mn >= INT_INF) break;
                lo = std::max<i64>(mn / delta * delta, hi);  // the next occupied band
                continue;
            }
            ++bands;
            i64 fsize = cnt;  // the round's frontier, all ranks
            for (;;) {  // light rounds until no rank has a frontier
                // a big round may pull (the gate keeps the counts off small rounds; every rank
                // sees the same fsize)
                bool lpulled = false;
                if (light_pull_ok && hi - lo <= map_w && fsize * 64 >= S.n) {
                    i64 lc[2] = {0, 0};
                    S.light_counts((int32_t)lo, (int32_t)hi, lc);
                    comm.allreduce(lc, 2, false, s);
                    if (lc[0] > 0 && (double)lc[0] * lpf > (double)lc[1]) {
                        i64 fm = S.frontier_min();  // (-1 on every rank alike: no bound)
                        if (fm >= 0) {
                            comm.allreduce(&fm, 1, true, s);
                            S.set_frontier_min(fm);
                        }
                        S.frontier_slice((int32_t)lo, (int32_t)hi);
                        if (S.world > 1) {
                            const size_t sl = S.member_bytes();
                            comm.allgather(static_cast<char*>(S.member_map()) + (size_t)S.rank * sl, S.member_map(),
                                           sl, s);
                        }
                        S.light_pull((int32_t)lo, (int32_t)hi);
                        lpulled = true;
                        ++lpulls;
                    }
                }
                if (!lpulled) exchange_apply(1, (int32_t)lo, (int32_t)hi);
                ++rounds;
                i64 nf = 0;
                if (dev) {
                    S.end_round_async();
                    comm.allgather_rows_dev(S.nf_dev(), 1, rows.data(), s);
                    for (int q = 0; q < S.world; ++q) nf += rows[(size_t)q];
                } else {
                    nf = S.end_round();
                    comm.allreduce(&nf, 1, false, s);
                }
                if (nf == 0) break;
                fsize = nf;
            }
            // heavy edges of the band's members: pulled by the unsettled vertices when those
            // have fewer heavy edges than pull_factor x the members' (v2's rule, §4.2), else pushed
            bool pulled = false;
            if (heavy_pull_ok && hi - lo <= 255) {  // (member offsets are bytes)
                i64 hc[2] = {0, 0};
                S.heavy_counts((int32_t)lo, (int32_t)hi, hc);
                comm.allreduce(hc, 2, false, s);
                if (hc[0] > 0 && (double)hc[1] < pf * (double)hc[0]) {
                    S.member_slice((int32_t)lo, (int32_t)hi);
                    if (S.world > 1) {
                        const size_t sl = S.member_bytes();
                        comm.allgather(static_cast<char*>(S.member_map()) + (size_t)S.rank * sl, S.member_map(), sl, s);
                    }
                    S.heavy_pull((int32_t)lo, (int32_t)hi);
                    pulled = true;
                    ++pulls;
                }
            }
            if (!pulled) exchange_apply(0, (int32_t)lo, (int32_t)hi);
            if (tail_on) {
                i64 ue = S.unsettled_edges((int32_t)hi);
                if (ue < 0) {
                    tail_on = false;  // (not supported: the same on every rank)
                } else {
                    comm.allreduce(&ue, 1, false, s);
                    if ((double)ue < tfrac * (double)all_edges) {
                        delta = tdelta;
                        S.set_delta(delta);
                        tail_on = false;
                        light_pull_ok = tail_light_ok;  // the tail's own light-pull rule
                        lpf = tlpf;
                        if (S.settled_map()) {  // everything below hi is settled from here on
                            S.settled_slice((int32_t)hi);
                            if (S.world > 1) {
                                const size_t sl = S.settled_bytes();
                                comm.allgather(static_cast<char*>(S.settled_map()) + (size_t)S.rank * sl,
                                               S.settled_map(), sl, s);
                            }
                        }
                    }
                }
            }
            lo = hi;
        }
        comm.sync(s);
        const double t1 = now_ms();
        i64 rc[2];
        S.reach(rc);
        comm.allreduce(rc, 2, false, s);
        if (st) {
            *st = pj_part_stats{};
            st->solve_ms = t1 - t0;
            st->levels = bands;
            st->bands = bands;
            st->rounds = rounds;
            st->delta = delta0;
            st->reached = rc[0];
            st->reached_edges = rc[1];
            st->sent = sent;
            st->heavy_pulls = (int32_t)pulls;
            st->bu_levels = lpulls;  // (delta-stepping: light rounds run as pulls)
        }
    });
}

}  // namespace pj
