// The multi-rank gather protocol of include/rt2.h ("Multi-GPU"), separated
// from its transport so that the control flow — who issues which collective
// when a rank fails locally — is the same code under RCCL (rt2_comm.hip) and
// under the thread-based fake transport of tests/comm_protocol/ (CPU test of
// every failure site, world sizes 2 and 3).  Host C++ only: no HIP, no RCCL.
//
// The rule: every rank issues the same collectives in the same order,
// whatever happened locally; a rank-local failure is decided by an agreement
// step (a 2-int allreduce(max) whose result every rank reads on the host)
// before any gather, so all ranks return < 0 together.  A rank that cannot
// take part in an agreement at all (its communicator was aborted, or the
// agreement's own copy/allreduce/wait fails) aborts and returns; its peers
// are then stuck in that agreement until their watchdog — the transport's
// wait with a deadline (RT2_COMM_TIMEOUT_S) — aborts their communicator, so
// every rank returns < 0 within the timeout instead of hanging.
//
// Transport T:
//   bool usable()                     the communicator can issue collectives
//   int  agree(int32_t v[2])          allreduce(max) of v in place, waited for
//                                     under the watchdog; on failure it has
//                                     aborted the communicator and returns -1
//   void abort(const std::string&)    make the communicator unusable
//   bool fault(const char* site)      fault injection (RT2_FAULT_AT), else false
#pragma once

#include <cstdint>
#include <string>

namespace rt2p {

// rt2_gather_slabs: prepare (this rank's checks, padding, receive buffer) ->
// agreement -> the one gather -> finish (the root's un-interleave).
// `prepare` returns 0 or sets err; `gather` issues the collective (its
// failure aborts: the peers may already be inside it); `finish` is local.
template <class T, class Prepare, class Gather, class Finish>
int gather_slabs(T& t, Prepare&& prepare, Gather&& gather, Finish&& finish, std::string& err) {
    if (!t.usable()) {
        err = "the communicator was aborted after an earlier failure";
        return -1;
    }
    int lrc = t.fault("gather.prepare") ? (err = "injected fault at gather.prepare", -1) : prepare(err);
    int32_t v[2] = {lrc != 0 ? 1 : 0, 0};
    if (t.agree(v) != 0) {
        err = "agreement before the gather failed: " + err;
        return -1;
    }
    if (v[0]) {
        if (lrc == 0) err = "a peer rank failed before the gather";
        return -1;
    }
    if (t.fault("gather.issue") || gather() != 0) {
        t.abort("the gather could not be issued");
        err = "the gather could not be issued (communicator aborted)";
        return -1;
    }
    return finish(err);
}

// rt2_render_host_gather: agreement 1 (local argument checks + whether any
// rank wants the 8-bit sums) -> local render -> agreement 2 (every rank
// rendered) -> the gathers (colour, then 8-bit when agreed) -> finish (the
// root's copies out, then a wait under the watchdog).
template <class T, class Render, class Gathers, class Finish>
int render_gather(T& t, bool args_ok, const std::string& args_err, bool want_rgb8, Render&& render, Gathers&& gathers,
                  Finish&& finish, std::string& err) {
    if (!t.usable()) {
        err = "the communicator was aborted after an earlier failure";
        return -1;
    }
    if (t.fault("check")) args_ok = false;
    int32_t v[2] = {args_ok ? 0 : 1, want_rgb8 ? 1 : 0};
    if (t.agree(v) != 0) {
        err = "agreement 1 failed";
        return -1;
    }
    if (v[0]) {
        err = args_ok ? std::string("a peer rank failed") : (args_err.empty() ? "injected fault at check" : args_err);
        return -1;
    }
    const bool rgb8 = v[1] != 0;
    std::string lerr;
    const int lrc = t.fault("render") ? (lerr = "injected fault at render", -1) : render(rgb8, lerr);
    v[0] = lrc != 0 ? 1 : 0;
    v[1] = 0;
    if (t.agree(v) != 0) {
        err = "agreement 2 failed" + (lerr.empty() ? std::string() : ": " + lerr);
        return -1;
    }
    if (v[0]) {
        err = lrc != 0 ? lerr : std::string("a peer rank failed");
        return -1;
    }
    if (t.fault("gather.issue") || gathers(rgb8) != 0) {
        t.abort("a gather could not be issued");
        err = "a gather could not be issued (communicator aborted)";
        return -1;
    }
    return finish(rgb8, err);
}

}  // namespace rt2p
