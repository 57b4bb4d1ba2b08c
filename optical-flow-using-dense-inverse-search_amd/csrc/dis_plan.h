// dis_plan.h -- the stream plan of a batch call (fork into the sub-batch
// streams, the stages of every sub-batch, join back into the caller's stream)
// as data, and the rules a plan must keep to be captured into a HIP graph.
// Host-only: dis_runtime.hip executes the plan (eagerly or under
// hipStreamBeginCapture); dis_plan.cpp builds and checks it, and exports both
// through the C-ABI so a CPU test can check the product's plans.
#pragma once

#include <string>
#include <vector>

namespace dis {

// stream 0 = the caller's (capture origin) stream, 1 + k = sub-batch stream k;
// event 0 = the fork event, 1 + k = sub-batch k's join event
enum PlanKind { kOpRecord = 0, kOpWait = 1, kOpWork = 2 };
struct PlanOp {
    int kind;
    int stream;
    int event;  // record / wait
    int stage;  // work: index into the call's stage list
};

// The product's plan for `S` >= 2 sub-batches and `nstages` stages: record
// the fork on the origin, every sub-batch stream waits on it, the stages
// stage-major (every sub-batch's stage t before any stage t + 1), then each
// sub-batch stream records its join event and the origin waits on it.
std::vector<PlanOp> batch_plan(int S, int nstages);

// Whether `ops` can be captured from the origin stream (empty string) or what
// breaks the rules, each measured on HIP 7.2 / gfx950 (tools/capture_probe.hip,
// tools/repro_sibling_capture.sh):
//  R1 a stream joins the capture by waiting on an event recorded in it (fork);
//  R2 every wait is on an event recorded earlier in the same capture: a wait
//     on an event recorded before the capture began is accepted and silently
//     dropped from the graph (the dependency is lost, probe mode 3);
//  R3 work and records only on streams in the capture;
//  R4 at the end every stream that joined has been joined back: all of its
//     operations happen before the origin's last one. An unjoined stream makes
//     hipStreamEndCapture fail with hipErrorStreamCaptureUnjoined, leaves that
//     stream in capture mode (a later synchronise on it fails, mode 9) and
//     writes a non-null handle that is not a graph (instantiating it crashed
//     the probe's process; destroying it returns hipErrorIllegalState);
//  R5 no sibling edge: a sub-batch stream waits only on events the origin
//     recorded. The product's capture with one mid-call barrier between the
//     sub-batch streams SIGSEGVs inside hipStreamEndCapture, with the join
//     events reused or with events of its own, while the eager call runs and
//     small probe graphs of the same shape capture fine (modes 2, 7, 10-13) --
//     the r05 crash (its merged finest launch waited on sibling events).
std::string check_capture_plan(const PlanOp* ops, int n, int nstreams, int nevents);

}  // namespace dis
