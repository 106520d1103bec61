// replay — re-issues, from ONE thread, the stream/event/copy/kernel calls a
// capture made (an op file extracted from an AMD_LOG_LEVEL=4 log by
// tools/capture/extract_ops.py), with stand-in streams, events, buffers and
// a dummy kernel.  A crash here reproduces the hipStreamEndCapture crash
// outside ftar; dropping ops (argv[2] = kinds to drop, e.g. "m" = memcpys,
// "k" = kernels) bisects it.
//   ops: B s | R e s | W s e | M s | K s | E s
// argv[3] = k: stop after the k-th op, join every stream used so far into the
// origin stream and end the capture there (the shortest crashing prefix).
// argv[4] = i: skip the i-th op (which ops the crash needs).
// drop kind 'p' (prune): simulate the capture's dependency
// sets -- per stream the nodes its next captured op will depend on, per event
// the set its record captured -- and skip every wait that adds nothing: all of
// the event's nodes are already the waiting stream's dependencies or their
// ancestors (a stream's FIRST wait, which brings it into the capture, is
// always kept).  If the pruned replay ends its capture where the full one
// crashes, redundant ancestor edges are what the runtime cannot handle.
// drop kind 'l' (leaves): keep every op, but after each wait ask the runtime
// for the stream's capture dependencies (hipStreamGetCaptureInfo_v2) and set
// them to their leaves (hipStreamUpdateCaptureDependencies): no node then
// depends on a node and that node's ancestor at once.  'v' prints the
// runtime's dependency count after every wait.
// drop kind 'f' (flat forks): right after the capture begins, every stream of
// the op file forks from the origin stream (one event recorded there, waited
// on by all), so no stream joins the capture through another forked stream;
// the file's own fork waits then become ordinary cross-stream waits and the
// dependencies stay the same (the begin event carries none).
// drop kind 'n' (node first): right after the capture begins, one tiny kernel
// node on the origin stream, so no event of the capture is recorded before the
// graph has a node (forks from an empty capture are the one shape every
// crashing log shares).
// drop kind 'a' (acyclic; diagnostic, changes the dependencies): skip every
// cross-stream wait that would close a cycle in the relation "stream W waited
// on an event recorded on stream R" (edge R -> W) -- e.g. the comm and reduce
// streams waiting on each other in turn.  Forks (a stream's first wait) and
// joins (a stream waiting on a stream it forked, directly or not) are kept.
// A capture that then ends says the runtime cannot end captures whose
// streams waited on each other both ways.
#include <hip/hip_runtime.h>

#include <set>
#include <vector>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "line %d: %s: %s\n", lineno, #x, hipGetErrorString(e_));            \
      exit(2);                                                                             \
    }                                                                                      \
  } while (0)

__global__ void touch(float* p) { p[threadIdx.x] += 1.0f; }

int main(int argc, char** argv) {
  std::ifstream in(argv[1]);
  const std::string drop = argc > 2 ? argv[2] : "";
  const int stop_after = argc > 3 ? atoi(argv[3]) : -1;
  const int skip = argc > 4 ? atoi(argv[4]) : -1;
  std::string origin;
  std::map<std::string, hipStream_t> streams;
  std::map<std::string, hipEvent_t> events;
  int lineno = 0;
  float *a, *b;
  CK(hipMalloc(&a, 1 << 20));
  CK(hipMalloc(&b, 1 << 20));
  auto S = [&](const std::string& k) {
    if (!streams.count(k)) CK(hipStreamCreateWithFlags(&streams[k], hipStreamNonBlocking));
    return streams[k];
  };
  auto E = [&](const std::string& k) {
    if (!events.count(k)) CK(hipEventCreateWithFlags(&events[k], hipEventDisableTiming));
    return events[k];
  };
  const bool leaves_only = drop.find('l') != std::string::npos, verbose = drop.find('v') != std::string::npos;
  int leaf_removed = 0;
  // the stream's capture dependencies reduced to their leaves; returns how many were dropped
  auto leaf_reduce = [&](hipStream_t st, const std::string& name) -> int {
    hipStreamCaptureStatus cs;
    const hipGraphNode_t* deps = nullptr;
    size_t nd = 0;
    CK(hipStreamGetCaptureInfo_v2(st, &cs, nullptr, nullptr, &deps, &nd));
    if (verbose) fprintf(stderr, "replay: %s has %zu capture dependencies\n", name.c_str(), nd);
    if (!leaves_only || cs != hipStreamCaptureStatusActive || nd < 2) return 0;
    std::vector<hipGraphNode_t> d(deps, deps + nd);
    std::set<hipGraphNode_t> anc;  // strict ancestors of the set's members
    std::vector<hipGraphNode_t> st_(d.begin(), d.end());
    while (!st_.empty()) {
      hipGraphNode_t v = st_.back();
      st_.pop_back();
      size_t np = 0;
      CK(hipGraphNodeGetDependencies(v, nullptr, &np));
      std::vector<hipGraphNode_t> ps(np);
      if (np) CK(hipGraphNodeGetDependencies(v, ps.data(), &np));
      for (hipGraphNode_t u : ps)
        if (anc.insert(u).second) st_.push_back(u);
    }
    std::vector<hipGraphNode_t> keep;
    std::set<hipGraphNode_t> seen;
    for (hipGraphNode_t v : d)
      if (!anc.count(v) && seen.insert(v).second) keep.push_back(v);
    if (keep.size() == nd) return 0;
    CK(hipStreamUpdateCaptureDependencies(st, keep.data(), keep.size(), hipStreamSetCaptureDependencies));
    return (int)(nd - keep.size());
  };
  // prune-mode simulation of the capture graph
  const bool prune = drop.find('p') != std::string::npos;
  std::vector<std::set<int>> node_deps;           // captured work nodes (M, K) and their dependencies
  std::map<std::string, std::set<int>> sdeps;     // stream -> dependency set of its next captured op
  std::map<std::string, bool> scap;               // stream is part of the capture
  std::map<std::string, std::set<int>> edeps;     // event -> the set its record captured
  std::map<std::string, bool> ecap;
  int pruned = 0, kept_waits = 0;
  auto closure = [&](const std::set<int>& from) {  // the set and all its ancestors
    std::set<int> out;
    std::vector<int> st(from.begin(), from.end());
    while (!st.empty()) {
      const int v = st.back();
      st.pop_back();
      if (!out.insert(v).second) continue;
      for (int d : node_deps[v]) st.push_back(d);
    }
    return out;
  };
  const bool flat = drop.find('f') != std::string::npos, acyclic = drop.find('a') != std::string::npos;
  std::map<std::string, std::string> erec;                 // event -> stream it was recorded on
  std::map<std::string, std::set<std::string>> waited_by;  // R -> {W}: W waited on an event of R
  int cyc = 0;
  std::map<std::string, std::string> fork_parent;  // stream -> the stream whose event brought it into the capture
  auto forked_from = [&](const std::string& s, std::string r) {  // is s an ancestor of r in the fork tree
    while (fork_parent.count(r)) {
      r = fork_parent[r];
      if (r == s) return true;
    }
    return false;
  };
  auto reaches = [&](const std::string& from, const std::string& to) {
    std::set<std::string> seen;
    std::vector<std::string> st{from};
    while (!st.empty()) {
      std::string v = st.back();
      st.pop_back();
      if (v == to) return true;
      if (!seen.insert(v).second) continue;
      for (const std::string& w : waited_by[v]) st.push_back(w);
    }
    return false;
  };
  std::vector<std::string> all_streams;  // every stream the file names, for 'f'
  {
    std::ifstream pre(argv[1]);
    std::string l2;
    std::set<std::string> seen;
    while (std::getline(pre, l2)) {
      std::istringstream ls(l2);
      std::string op, x, y;
      ls >> op >> x >> y;
      const std::string st = op == "R" ? y : (op == "W" || op == "M" || op == "K" || op == "B" || op == "E") ? x : "";
      if (!st.empty() && seen.insert(st).second) all_streams.push_back(st);
    }
  }
  std::string line;
  int n = 0;
  while (std::getline(in, line)) {
    ++lineno;
    std::istringstream ls(line);
    std::string op, x, y;
    ls >> op >> x >> y;
    if (!op.empty() && drop.find(op[0] | 0x20) != std::string::npos && op != "B" && op != "E") continue;
    if (op != "B" && op != "E" && stop_after >= 0 && n >= stop_after) {
      // join everything used so far into the origin and end there
      for (auto& kv : streams) {
        if (kv.first == origin) continue;
        hipEvent_t j;
        CK(hipEventCreateWithFlags(&j, hipEventDisableTiming));
        CK(hipEventRecord(j, kv.second));
        CK(hipStreamWaitEvent(streams[origin], j, 0));
      }
      op = "E";
      x = origin;
    }
    if (op != "B" && op != "E" && n == skip) {
      ++n;
      continue;
    }
    if (op == "B") {
      origin = x;
      scap[x] = true;
      sdeps[x].clear();
      CK(hipStreamBeginCapture(S(x), hipStreamCaptureModeRelaxed));
      if (drop.find('n') != std::string::npos) {
        touch<<<1, 64, 0, S(x)>>>(a);
        node_deps.push_back(sdeps[x]);
        sdeps[x] = {(int)node_deps.size() - 1};
        fprintf(stderr, "replay: a kernel node on the origin before any record\n");
      }
      if (flat) {
        hipEvent_t root;
        CK(hipEventCreateWithFlags(&root, hipEventDisableTiming));
        CK(hipEventRecord(root, S(x)));
        int forked = 0;
        for (const std::string& st : all_streams)
          if (st != x) {
            CK(hipStreamWaitEvent(S(st), root, 0));
            scap[st] = true;
            ++forked;
          }
        fprintf(stderr, "replay: %d streams forked from the origin at capture begin\n", forked);
      }
    }
    else if (op == "R") {
      erec[x] = y;
      edeps[x] = sdeps[y];
      ecap[x] = scap[y];
      CK(hipEventRecord(E(x), S(y)));
    }
    else if (op == "W") {
      const std::string rec = erec[y];
      const bool fork = ecap[y] && !scap[x], join = forked_from(x, rec);
      if (fork) fork_parent[x] = rec;
      if (acyclic && !fork && !join && !rec.empty() && rec != x && reaches(x, rec)) {
        ++cyc;
        fprintf(stderr, "replay: skipped op %d (W %s on an event of %s: closes a wait cycle)\n", n, x.c_str(),
                rec.c_str());
        ++n;
        continue;
      }
      if (!rec.empty() && rec != x) waited_by[rec].insert(x);
      if (ecap[y] && !scap[x]) {  // the fork: the stream joins the capture
        scap[x] = true;
        sdeps[x] = edeps[y];
      } else if (ecap[y]) {
        const std::set<int> have = closure(sdeps[x]);
        bool adds = false;
        for (int v : edeps[y]) adds = adds || !have.count(v);
        if (prune && !adds) {
          ++pruned;
          fprintf(stderr, "replay: pruned op %d (W %s %s: adds nothing)\n", n, x.c_str(), y.c_str());
          ++n;
          continue;
        }
        for (int v : edeps[y]) sdeps[x].insert(v);
      }
      ++kept_waits;
      CK(hipStreamWaitEvent(S(x), E(y), 0));
      leaf_removed += leaf_reduce(S(x), x);
    }
    else if (op == "M" || op == "K") {
      node_deps.push_back(sdeps[x]);
      sdeps[x] = {(int)node_deps.size() - 1};
      if (op == "M") CK(hipMemcpyAsync(b, a, 256, hipMemcpyDeviceToDevice, S(x)));
      else touch<<<1, 64, 0, S(x)>>>(a);
    }
    else if (op == "E") {
      hipGraph_t g;
      fprintf(stderr, "replay: %d ops, %d waits kept, %d pruned as redundant, %d ancestor dependencies removed, "
              "%d cycle-closing waits skipped; ending the capture\n", n, kept_waits, pruned, leaf_removed, cyc);
      CK(hipStreamEndCapture(S(x), &g));
      size_t nodes = 0;
      CK(hipGraphGetNodes(g, nullptr, &nodes));
      printf("replay ok: %zu nodes (mode '%s'; %d waits kept, %d pruned, %d ancestor dependencies removed)\n", nodes,
             drop.c_str(), kept_waits, pruned, leaf_removed);
      return 0;
    }
    ++n;
  }
  fprintf(stderr, "no end of capture in the op file\n");
  return 1;
}
