// dis_plan.cpp -- batch-call stream plans and their capture rules (dis_plan.h).
#include "dis_plan.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "dis_abi.h"

namespace dis {

dis_status set_error(dis_status s, const std::string& msg);  // dis_runtime.hip

std::vector<PlanOp> batch_plan(int S, int nstages)
{
    std::vector<PlanOp> ops;
    ops.push_back({kOpRecord, 0, 0, -1});
    for (int k = 0; k < S; ++k) ops.push_back({kOpWait, 1 + k, 0, -1});
    for (int t = 0; t < nstages; ++t)
        for (int k = 0; k < S; ++k) ops.push_back({kOpWork, 1 + k, -1, t});
    for (int k = 0; k < S; ++k) {
        ops.push_back({kOpRecord, 1 + k, 1 + k, -1});
        ops.push_back({kOpWait, 0, 1 + k, -1});
    }
    return ops;
}

std::string check_capture_plan(const PlanOp* ops, int n, int nstreams, int nevents)
{
    if (nstreams < 1 || nevents < 0 || n < 0) return "bad plan dimensions";
    char b[176];
    const size_t S = (size_t)nstreams;
    std::vector<char> member(S, 0);
    std::vector<int> rec_op((size_t)nevents, -1);  // op that last recorded the event in this capture
    std::vector<int> last_op(S, -1);               // the stream's last op
    // vector clocks: vc[i][x] = the latest op of stream x that happens before
    // (or is) op i, -1 if none
    std::vector<std::vector<int>> vc((size_t)n, std::vector<int>(S, -1));
    member[0] = 1;
    for (int i = 0; i < n; ++i) {
        const PlanOp& o = ops[i];
        if (o.stream < 0 || o.stream >= nstreams) return "op " + std::to_string(i) + ": stream out of range";
        if ((o.kind == kOpRecord || o.kind == kOpWait) && (o.event < 0 || o.event >= nevents))
            return "op " + std::to_string(i) + ": event out of range";
        if (o.kind != kOpRecord && o.kind != kOpWait && o.kind != kOpWork)
            return "op " + std::to_string(i) + ": unknown kind";
        if (last_op[o.stream] >= 0) vc[i] = vc[last_op[o.stream]];
        if (o.kind == kOpWait) {
            const int r = rec_op[o.event];
            if (r < 0) {
                std::snprintf(b, sizeof b,
                              "op %d: stream %d waits on event %d, which was not recorded in this capture (R2)", i,
                              o.stream, o.event);
                return b;
            }
            if (o.stream != 0 && ops[r].stream != 0) {
                std::snprintf(b, sizeof b,
                              "op %d: sub-batch stream %d waits on event %d of sub-batch stream %d: a sibling edge (R5)",
                              i, o.stream, o.event, ops[r].stream);
                return b;
            }
            for (size_t x = 0; x < S; ++x) vc[i][x] = std::max(vc[i][x], vc[r][x]);
            member[o.stream] = 1;  // R1
        } else if (!member[o.stream]) {
            std::snprintf(b, sizeof b, "op %d: %s on stream %d, which is not in the capture (R3)", i,
                          o.kind == kOpRecord ? "record" : "work", o.stream);
            return b;
        }
        if (o.kind == kOpRecord) rec_op[o.event] = i;
        vc[i][o.stream] = i;
        last_op[o.stream] = i;
    }
    const int end = last_op[0];
    for (size_t x = 1; x < S; ++x) {
        if (!member[x] || last_op[x] < 0) continue;
        if (end < 0 || vc[end][x] < last_op[x]) {
            std::snprintf(b, sizeof b,
                          "stream %d is not joined back: its op %d does not happen before the origin's last op (R4)",
                          (int)x, last_op[x]);
            return b;
        }
    }
    return std::string();
}

}  // namespace dis

extern "C" {

dis_status dis_batch_stream_plan(int nsub, int nstages, int* ops, int capacity, int* count)
{
    if (nsub < 2 || nsub > 8 || nstages < 1 || !count) return dis::set_error(DIS_ERR_INVALID_ARGUMENT, "bad argument");
    const std::vector<dis::PlanOp> p = dis::batch_plan(nsub, nstages);
    *count = (int)p.size();
    if (!ops) return DIS_OK;
    if (capacity < (int)p.size()) return dis::set_error(DIS_ERR_INVALID_ARGUMENT, "capacity too small");
    for (size_t i = 0; i < p.size(); ++i) {
        ops[4 * i] = p[i].kind;
        ops[4 * i + 1] = p[i].stream;
        ops[4 * i + 2] = p[i].event;
        ops[4 * i + 3] = p[i].stage;
    }
    return DIS_OK;
}

dis_status dis_check_stream_plan(const int* ops, int nops, int nstreams, int nevents)
{
    if (!ops || nops < 0) return dis::set_error(DIS_ERR_INVALID_ARGUMENT, "bad argument");
    std::vector<dis::PlanOp> p((size_t)nops);
    for (int i = 0; i < nops; ++i) p[i] = {ops[4 * i], ops[4 * i + 1], ops[4 * i + 2], ops[4 * i + 3]};
    const std::string why = dis::check_capture_plan(p.data(), nops, nstreams, nevents);
    if (!why.empty()) return dis::set_error(DIS_ERR_UNSUPPORTED, why);
    return DIS_OK;
}

}  // extern "C"
