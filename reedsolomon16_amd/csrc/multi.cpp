// Multi-device codec (rs_new_multi, multi.hpp): the byte-range split of
// SURVEY §8(e) behind the single-codec C-ABI, so a cgo caller holding one
// Encoder (reedsolomon.go:90-93) drives every GPU of the node.
//
// A call on the parent codec cuts every shard into the parts' 64-byte-granular
// byte ranges and hands part g its range on its own host worker thread, which
// runs the part's host pipeline (its own streams, staging slabs and tickets)
// on its device.  The threads only issue HIP calls: the data never leaves the
// caller's rows except over each device's own PCIe link.  Asynchronous calls
// return one parent ticket that maps to one ticket per part.
#include <condition_variable>
#include <deque>
#include <functional>
#include <future>
#include <memory>
#include <mutex>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/rs_mi355x.h"
#include "multi.hpp"

namespace rs {

void part_byte_range(uint64_t S, int g, int n, uint64_t &lo, uint64_t &hi) {
    const uint64_t blocks = S / 64, base = blocks / (uint64_t)n, extra = blocks % (uint64_t)n;
    const uint64_t ug = (uint64_t)g;
    lo = ug * base + (ug < extra ? ug : extra);
    hi = lo + base + (ug < extra ? 1 : 0);
    lo *= 64;
    hi *= 64;
}

namespace {

// One host thread per part: jobs run in submission order, so a part's calls
// (and the tickets they queue) keep the order of the parent's calls.
class Worker {
  public:
    Worker() : th_([this] { loop(); }) {}
    ~Worker() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
        }
        cv_.notify_one();
        th_.join();
    }
    std::future<int> submit(std::function<int()> fn) {
        std::packaged_task<int()> t(std::move(fn));
        std::future<int> f = t.get_future();
        {
            std::lock_guard<std::mutex> lk(m_);
            q_.push_back(std::move(t));
        }
        cv_.notify_one();
        return f;
    }

  private:
    void loop() {
        for (;;) {
            std::packaged_task<int()> t;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
                if (q_.empty()) return;  // stop_ and drained
                t = std::move(q_.front());
                q_.pop_front();
            }
            t();
        }
    }
    std::mutex m_;
    std::condition_variable cv_;
    std::deque<std::packaged_task<int()>> q_;
    bool stop_ = false;
    std::thread th_;  // last: starts after the members it uses exist
};

}  // namespace

struct Multi {
    std::vector<rs_codec *> parts;
    std::vector<int> devices;
    std::vector<std::unique_ptr<Worker>> workers;
    // parent tickets: slot t % kTickets holds ticket t's per-part tickets
    // (part index, part ticket) until a later ticket takes the slot
    static constexpr int kTickets = 64;
    struct Slot {
        uint64_t id = 0;
        HostOp op = HostOp::Encode;
        std::vector<std::pair<int, uint64_t>> subs;
    };
    std::mutex tmu;
    Slot slots[kTickets];
    uint64_t next = 1;
};

Multi *multi_create(std::vector<rs_codec *> parts, std::vector<int> devices) {
    Multi *m = new (std::nothrow) Multi();
    if (!m) return nullptr;
    try {  // thread creation can fail: no exception crosses the C-ABI
        for (size_t g = 0; g < parts.size(); g++) m->workers.emplace_back(new Worker());
    } catch (...) {
        delete m;  // joins the workers already started; the caller still owns the parts
        return nullptr;
    }
    m->parts = std::move(parts);
    m->devices = std::move(devices);
    return m;
}

void multi_destroy(Multi *m) {
    if (!m) return;
    m->workers.clear();  // joins the threads (every job has completed: calls wait for theirs)
    for (rs_codec *p : m->parts) rs_free(p);
    delete m;
}

int multi_count(const Multi *m) { return (int)m->parts.size(); }

rs_codec *multi_part(Multi *m, int g, int *device) {
    if (device) *device = m->devices[g];
    return m->parts[g];
}

int multi_host(Multi *m, rs_codec *parent, HostOp op, uint8_t *const *shards, uint64_t S,
               const std::vector<uint8_t> &present, bool recover_all, int *ok, uint64_t *ticket) {
    const int n = (int)m->parts.size(), total = rs_total_shards(parent);
    ElExt el;
    if (op == HostOp::Reconstruct)  // once for every part, keyed on the full shard size
        if (int e = parent_error_locators(parent, present, recover_all, S, el)) return e;
    std::vector<std::vector<uint8_t *>> rows(n);
    std::vector<uint64_t> sub(n, 0);
    std::vector<int> oks(n, 1), active;
    std::vector<std::future<int>> fut;
    for (int g = 0; g < n; g++) {
        uint64_t lo, hi;
        part_byte_range(S, g, n, lo, hi);
        if (hi == lo) continue;  // fewer 64-byte blocks than parts
        rows[g].resize(total);
        for (int i = 0; i < total; i++) rows[g][i] = shards[i] ? shards[i] + lo : nullptr;
        const uint64_t w = hi - lo;
        active.push_back(g);
        fut.push_back(m->workers[g]->submit([&, g, w] {
            return part_host_call(m->parts[g], op, rows[g].data(), w, present, recover_all,
                                  op == HostOp::Verify ? &oks[g] : nullptr, ticket ? &sub[g] : nullptr,
                                  op == HostOp::Reconstruct ? &el : nullptr);
        }));
    }
    int err = RS_OK;
    for (auto &f : fut) {  // every part has returned before the parent does (rows, el live on this frame)
        const int e = f.get();
        if (e && !err) err = e;
    }
    if (err) {
        // parts that queued work still write the caller's rows: finish it
        // before reporting the error, so the caller may release them
        if (ticket)
            for (int g : active)
                if (sub[g]) (void)rs_ticket_wait(m->parts[g], sub[g]);
        return err;
    }
    if (ok) {
        *ok = 1;
        for (int g : active) *ok = *ok && oks[g];
    }
    if (ticket) {
        std::lock_guard<std::mutex> lk(m->tmu);
        const uint64_t id = m->next++;
        Multi::Slot &s = m->slots[id % Multi::kTickets];
        s.id = id;
        s.op = op;
        s.subs.clear();
        for (int g : active)
            if (sub[g]) s.subs.emplace_back(g, sub[g]);
        *ticket = id;
    }
    return RS_OK;
}

namespace {
// The per-part tickets behind parent ticket t.  A slot a later ticket has
// taken holds that later ticket's parts, whose work each part queued after
// t's (same streams, FIFO workers): waiting on them also covers t.
int ticket_subs(Multi *m, uint64_t t, std::vector<std::pair<int, uint64_t>> &subs) {
    std::lock_guard<std::mutex> lk(m->tmu);
    if (t >= m->next) return RS_ERR_INVALID_ARG;
    subs = m->slots[t % Multi::kTickets].subs;
    return RS_OK;
}
}  // namespace

int multi_ticket_wait(Multi *m, uint64_t t) {
    if (t == 0) return RS_OK;  // no work was queued
    std::vector<std::pair<int, uint64_t>> subs;
    if (int e = ticket_subs(m, t, subs)) return e;
    for (auto &s : subs)
        if (int e = rs_ticket_wait(m->parts[s.first], s.second)) return e;
    return RS_OK;
}

int multi_ticket_query(Multi *m, uint64_t t, int *done) {
    *done = 1;
    if (t == 0) return RS_OK;
    std::vector<std::pair<int, uint64_t>> subs;
    if (int e = ticket_subs(m, t, subs)) return e;
    for (auto &s : subs) {
        int d = 0;
        if (int e = rs_ticket_query(m->parts[s.first], s.second, &d)) return e;
        if (!d) {
            *done = 0;
            return RS_OK;
        }
    }
    return RS_OK;
}

// Verify's only reduction: the AND of the parts' verdicts, on the host.
int multi_verify_result(Multi *m, uint64_t t, int *ok) {
    *ok = 0;
    std::vector<std::pair<int, uint64_t>> subs;
    {
        std::lock_guard<std::mutex> lk(m->tmu);
        const Multi::Slot &s = m->slots[t % Multi::kTickets];
        if (t == 0 || s.id != t || s.op != HostOp::Verify) return RS_ERR_INVALID_ARG;
        subs = s.subs;
    }
    int all = 1;
    for (auto &s : subs) {
        int o = 0;
        if (int e = rs_verify_result(m->parts[s.first], s.second, &o)) return e;
        all = all && o;
    }
    *ok = all;
    return RS_OK;
}

int multi_set_host_segment(Multi *m, size_t bytes) {
    for (rs_codec *p : m->parts)
        if (int e = rs_set_host_segment(p, bytes)) return e;
    return RS_OK;
}

}  // namespace rs
