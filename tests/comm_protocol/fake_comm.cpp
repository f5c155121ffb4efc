// CPU test of the multi-rank gather protocol (raytracing2-fork_amd/csrc/device/
// rt2_comm_protocol.h, the code rt2_comm.hip runs under RCCL): N ranks as
// threads over a fake transport whose collectives are rendezvous with a
// deadline, like the RCCL transport's watchdog.  For every failure site and
// failing rank it checks that every rank returns < 0 within the deadline (no
// hang), that no gather is issued after a failure the agreement caught, and
// that a clean run gathers on every rank.  Prints one JSON object per case.
//
//   g++ -std=c++17 -O1 -pthread -I<repo>/raytracing2-fork_amd/csrc/device fake_comm.cpp
#include <algorithm>
#include <chrono>
#include <climits>
#include <condition_variable>
#include <cstdio>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "rt2_comm_protocol.h"

namespace {

constexpr double kTimeout = 0.5;  // the fake's RT2_COMM_TIMEOUT_S

// One communicator shared by the rank threads: collective k is a rendezvous
// of all ranks (values max-reduced); a rank that arrives waits until every
// rank has arrived or the deadline passes.
struct World {
    int n;
    std::mutex m;
    std::condition_variable cv;
    struct Slot {
        int arrived = 0;
        int32_t v[2] = {INT32_MIN, INT32_MIN};
    };
    std::map<int, Slot> slots;
    int gathers_issued = 0;
    explicit World(int n_) : n(n_) {}
    // 0 when every rank arrived, -1 at the deadline
    int rendezvous(int k, int32_t* v) {
        std::unique_lock<std::mutex> lk(m);
        Slot& s = slots[k];
        if (v) {
            s.v[0] = std::max(s.v[0], v[0]);
            s.v[1] = std::max(s.v[1], v[1]);
        }
        s.arrived++;
        cv.notify_all();
        const bool ok = cv.wait_for(lk, std::chrono::duration<double>(kTimeout), [&] { return s.arrived >= n; });
        if (!ok) return -1;
        if (v) {
            v[0] = s.v[0];
            v[1] = s.v[1];
        }
        return 0;
    }
};

struct FakeTransport {
    World* w;
    int rank;
    std::string site;
    int fault_rank;
    int seq = 0;  // collectives this rank has issued, in order (RCCL's ordering rule)
    bool aborted = false;
    bool usable() const { return !aborted; }
    bool fault(const char* s) const { return site == s && (fault_rank < 0 || fault_rank == rank); }
    void abort(const std::string&) { aborted = true; }
    int agree(int32_t v[2]) {
        if (!usable()) return -1;
        if (fault("agree.copy")) {  // this rank cannot take part in the agreement
            abort("copy");
            return -1;
        }
        if (w->rendezvous(seq++, v) != 0) {  // the watchdog's deadline
            abort("timeout");
            return -1;
        }
        return 0;
    }
    // a gather: issued now (asynchronous), completed by wait_gather
    int issue_gather() {
        std::lock_guard<std::mutex> lk(w->m);
        w->gathers_issued++;
        return 0;
    }
    int wait_gather() {
        if (w->rendezvous(seq++, nullptr) != 0) {
            abort("timeout");
            return -1;
        }
        return 0;
    }
};

struct Result {
    int rc;
    double seconds;
};

// proto 0: rt2_gather_slabs (asynchronous: the caller waits for the gather
// later; the fake waits here so that a hang would show); proto 1:
// rt2_render_host_gather
#ifdef MUTANT_EARLY_RETURN
// mutant (tests/test_comm_protocol.py): a rank that fails locally returns
// before the agreement, as round 2's gather did; its peers then wait for the
// watchdog, which the checks above must flag
template <class T, class P, class G, class F>
int gather_slabs_mutant(T& t, P&& prepare, G&& gather, F&& finish, std::string& err) {
    if (t.fault("gather.prepare")) return -1;
    return rt2p::gather_slabs(t, prepare, gather, finish, err);
}
#define GATHER_SLABS gather_slabs_mutant
#else
#define GATHER_SLABS rt2p::gather_slabs
#endif

std::vector<Result> run(int proto, int n, const std::string& site, int fault_rank, int& gathers) {
    World w(n);
    std::vector<Result> res(n);
    std::vector<std::thread> th;
    for (int r = 0; r < n; r++) {
        th.emplace_back([&, r] {
            FakeTransport t{&w, r, site, fault_rank};
            std::string err;
            const auto t0 = std::chrono::steady_clock::now();
            int rc;
            if (proto == 0) {
                rc = GATHER_SLABS(
                    t, [&](std::string&) { return 0; }, [&] { return t.issue_gather(); },
                    [&](std::string&) { return 0; }, err);
                if (rc == 0 && t.wait_gather() != 0) rc = -2;  // the caller waits with rt2_comm_wait (its deadline)
            } else {
                rc = rt2p::render_gather(
                    t, true, "", r == 0, [&](bool, std::string&) { return 0; }, [&](bool) { return t.issue_gather(); },
                    [&](bool, std::string&) { return t.wait_gather(); }, err);
            }
            res[r] = {rc, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count()};
        });
    }
    for (auto& x : th) x.join();
    gathers = w.gathers_issued;
    return res;
}

}  // namespace

int main() {
    const char* sites[] = {"", "gather.prepare", "gather.issue", "check", "render", "agree.copy"};
    int bad = 0;
    for (int proto = 0; proto < 2; proto++) {
        for (int n : {2, 3}) {
            for (const char* site : sites) {
                const std::string s(site);
                if (proto == 0 && (s == "check" || s == "render")) continue;  // render_gather's sites
                if (proto == 1 && s == "gather.prepare") continue;            // gather_slabs' site
                for (int fr : s.empty() ? std::vector<int>{-1} : std::vector<int>{0, n - 1}) {
                    int gathers = 0;
                    const std::vector<Result> res = run(proto, n, s, fr, gathers);
                    double tmax = 0.0;
                    bool all_ok = true, all_fail = true;
                    for (const Result& x : res) {
                        tmax = std::max(tmax, x.seconds);
                        all_ok = all_ok && x.rc == 0;
                        all_fail = all_fail && x.rc < 0;
                    }
                    // clean: every rank succeeds and gathers; a fault: every rank
                    // fails, within the deadline (plus scheduling slack); a fault
                    // the agreement sees issues no gather anywhere
                    bool pass = s.empty() ? (all_ok && gathers == n) : all_fail;
                    pass = pass && tmax < 3 * kTimeout + 1.0;
                    // ... and without waiting for the watchdog: the agreement told every rank
                    const bool agreed = s == "gather.prepare" || s == "check" || s == "render";
                    if (agreed) pass = pass && gathers == 0 && tmax < 0.5 * kTimeout;
                    bad += !pass;
                    std::string rcs;
                    for (const Result& x : res) rcs += (rcs.empty() ? "" : ",") + std::to_string(x.rc);
                    std::printf("{\"proto\": \"%s\", \"n\": %d, \"site\": \"%s\", \"fault_rank\": %d, \"rc\": [%s], "
                                "\"gathers\": %d, \"seconds_max\": %.3f, \"pass\": %s}\n",
                                proto == 0 ? "gather_slabs" : "render_host_gather", n, site, fr, rcs.c_str(), gathers,
                                tmax, pass ? "true" : "false");
                }
            }
        }
    }
    return bad == 0 ? 0 : 1;
}
