// mcg-cg : command-line entry point.
//
// With NO arguments it behaves exactly like the reference binary
// (CUDACG.cu:41-366): solve the built-in 3x3 system on GPU 0 with maxit=2000,
// tol=1e-7 (absolute), print x one "%f\n" per entry, then "Success", exit 0.
// Any failure prints a one-line message to stdout (the reference prints
// everything through printf, CUDACG.cu:11) and exits 1; details go to stderr.
//
// Flags (all additive):
//   --problem demo|poisson2d|poisson3d|randspd|csr   --n N   --rows R --band W --density q --spread S
//   --scramble 0|1 (random-spd: P^T A P, a seeded random symmetric permutation)
//   --coef 0|1 (poisson2d/3d: 1 = variable coefficients from a seeded random conductivity field)
//   --matrix FILE.mtx (a user matrix, problem csr)  --rhs-file FILE (its b: Matrix Market array / one per line)
//   --rhs reference|random|ones  --seed S  --gpus P  --device gpu|cpu  --sim-ranks P (cpu)
//   --maxit M  --tol T  --rtol R (||r|| < R ||b||)  --check-every K  --fixed-iters K  --warmup W
//   --nnz-per-row m (random-spd: density = (m - 1) / (2 band))
//   --format csr|sell|sell16|sellc8  --no-overlap  --no-graph  --force-comm  --blocks-per-cu B
//   --comm single|dual (one RCCL communicator, one stream order (default) | two, halo on a side stream)
//   --spmv-variant 0|1|2|3|4
//   --recurrence two|single|pipelined  --pipe-rr K  --interleave auto|on|off  --window auto|on|off
//   --carry auto|on|off (line-carry stencil pass)  --halo-mode auto|window|allgather  --pmat auto|on|off
//   --fused-reduce auto|on|off  --watchdog SECONDS  --reserve-cus K
//   --checkpoint PREFIX  --checkpoint-every K  --resume PREFIX  --inject-nan-at K
//   --print-x auto|yes|no  --report text|json  --verify
//   --halo-transport auto|rccl  --allreduce auto|rccl|ipc  --transport-probe auto|off  --rehearse-ranks
// Multi-GPU runs use one host thread per GPU inside this process (no MPI in
// this image); the two RCCL unique ids are shared in memory.  At P > 1 each rank's
// communicator is wrapped in a PeerHaloComm that maps the other threads' halo
// buffers as plain pointers (peer access enabled), so the lean carries read their
// ghost lines from the neighbours' rows (halo_pull), and every rank's IPC
// all-reduce mailbox is mapped next to RCCL; the solver's transport probe picks
// the halo and the all-reduce at the first reset (--halo-transport rccl /
// --allreduce rccl: RCCL only).  --rehearse-ranks runs the P rank threads on
// GPU 0 with an in-process communicator (LocalComm) under the same wrapping: the
// real P-rank recurrence on one GPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "mcg/cg.hpp"
#include "mcg/check.hpp"
#include "mcg/comm.hpp"
#include "mcg/matrix.hpp"
#include "mcg/solver.hpp"

using namespace mcg;

namespace {

struct Args {
  ProblemSpec spec;
  CgOptions opt;
  int gpus = 1;
  bool cpu = false;
  int sim_ranks = 1;
  int fixed_iters = 0;
  int warmup = 0;
  double nnz_per_row = 0.0;  // random-spd: mean nonzeros per row (sets the density)
  std::string print_x = "auto";
  std::string report = "text";
  bool verify = false;
  bool rhs_set = false;
  bool format_set = false, recurrence_set = false;
  std::string resume;  // checkpoint prefix to resume from
  bool comm_single = true;  // --comm single (default): one RCCL communicator, collectives in one stream order
  std::string halo_transport = "auto";  // auto: peers mapped (in-kernel halo) | rccl
  std::string allreduce = "auto";       // auto: IPC mailboxes mapped, the probe decides | rccl | ipc
  bool rehearse = false;                // every rank thread on GPU 0 over LocalComm (one-GPU rehearsal)
  std::string matrix, rhs_file;  // user matrix (Matrix Market) and its right-hand side
  std::shared_ptr<HostMatrix> mat;
};

int tri(const std::string& v, const char* flag) {  // auto|on|off -> -1|1|0
  if (v == "auto" || v == "-1") return -1;
  if (v == "on" || v == "1" || v == "yes") return 1;
  if (v == "off" || v == "0" || v == "no") return 0;
  fail(std::string("invalid arguments: ") + flag + " " + v);
}

[[noreturn]] void usage_error(const std::string& m) { fail("invalid arguments: " + m); }

Args parse(int argc, char** argv) {
  Args a;
  auto need = [&](int& i) -> std::string {
    if (i + 1 >= argc) usage_error(std::string("missing value for ") + argv[i]);
    return argv[++i];
  };
  for (int i = 1; i < argc; ++i) {
    std::string f = argv[i];
    if (f == "--problem") {
      std::string v = need(i);
      if (v == "csr") a.spec.kind = ProblemKind::Csr;
      else a.spec.kind = parse_problem_kind(v);
    }
    else if (f == "--n") a.spec.N = std::stoll(need(i));
    else if (f == "--rows") a.spec.rows = std::stoll(need(i));
    else if (f == "--band") a.spec.band = std::stoll(need(i));
    else if (f == "--density") a.spec.density = std::stod(need(i));
    else if (f == "--spread") a.spec.spread = std::stoll(need(i));
    else if (f == "--scramble") a.spec.scramble = std::stoi(need(i));
    else if (f == "--coef") a.spec.coef = std::stoi(need(i));
    else if (f == "--matrix") a.matrix = need(i);
    else if (f == "--rhs-file") a.rhs_file = need(i);
    else if (f == "--halo-mode") {
      std::string v = need(i);
      a.opt.halo_mode = v == "window" ? 0 : (v == "allgather" ? 1 : tri(v, "--halo-mode"));
    }
    else if (f == "--pmat") a.opt.form.pmat = tri(need(i), "--pmat");
    else if (f == "--fused-reduce") a.opt.form.fused_reduce = tri(need(i), "--fused-reduce");
    else if (f == "--rhs") { a.spec.rhs = parse_rhs_kind(need(i)); a.rhs_set = true; }
    else if (f == "--seed") a.spec.seed = std::stoull(need(i));
    else if (f == "--gpus") a.gpus = std::stoi(need(i));
    else if (f == "--device") { std::string d = need(i); if (d == "cpu") a.cpu = true; else if (d != "gpu") usage_error(d); }
    else if (f == "--sim-ranks") a.sim_ranks = std::stoi(need(i));
    else if (f == "--maxit") a.opt.maxit = std::stoi(need(i));
    else if (f == "--tol") a.opt.tol = std::stod(need(i));
    else if (f == "--rtol") a.opt.rtol = std::stod(need(i));
    else if (f == "--watchdog") a.opt.watchdog_seconds = std::stod(need(i));
    else if (f == "--reserve-cus") a.opt.reserve_cus = std::stoi(need(i));
    else if (f == "--nnz-per-row") a.nnz_per_row = std::stod(need(i));
    else if (f == "--check-every") a.opt.check_every = std::stoi(need(i));
    else if (f == "--fixed-iters") a.fixed_iters = std::stoi(need(i));
    else if (f == "--warmup") a.warmup = std::stoi(need(i));
    else if (f == "--format") {
      std::string v = need(i);
      a.opt.format = (v == "sell" || v == "sell64") ? 1
                     : (v == "sell16" || v == "sell64-d16") ? 2
                     : (v == "sellc8" || v == "sell64-c8") ? 3
                                                            : 0;
      a.format_set = true;
    }
    else if (f == "--no-overlap") a.opt.overlap = false;
    else if (f == "--no-graph") a.opt.use_graph = false;
    else if (f == "--force-comm") a.opt.force_comm = true;
    else if (f == "--comm") {
      const std::string v = need(i);
      if (v != "single" && v != "dual") usage_error("--comm " + v);
      a.comm_single = v == "single";
    }
    else if (f == "--halo-transport") {
      a.halo_transport = need(i);
      if (a.halo_transport != "auto" && a.halo_transport != "rccl") usage_error("--halo-transport " + a.halo_transport);
    }
    else if (f == "--allreduce") {
      a.allreduce = need(i);
      if (a.allreduce != "auto" && a.allreduce != "rccl" && a.allreduce != "ipc") usage_error("--allreduce " + a.allreduce);
    }
    else if (f == "--transport-probe") a.opt.transport_probe = tri(need(i), "--transport-probe") == 0 ? 0 : -1;
    else if (f == "--rehearse-ranks") a.rehearse = true;
    else if (f == "--blocks-per-cu") a.opt.blocks_per_cu = std::stoi(need(i));
    else if (f == "--spmv-variant") a.opt.spmv_variant = std::stoi(need(i));
    else if (f == "--checkpoint") a.opt.checkpoint_path = need(i);
    else if (f == "--checkpoint-every") a.opt.checkpoint_every = std::stoi(need(i));
    else if (f == "--resume") a.resume = need(i);
    else if (f == "--inject-nan-at") a.opt.hooks.inject_nan_at = std::stoi(need(i));
    else if (f == "--recurrence") {
      std::string v = need(i);
      if (v == "auto" || v == "-1") a.opt.recurrence = -1;
      else if (v == "single" || v == "fused1" || v == "1") a.opt.recurrence = 1;
      else if (v == "two" || v == "0") a.opt.recurrence = 0;
      else if (v == "pipelined" || v == "2") a.opt.recurrence = 2;
      else usage_error("--recurrence " + v);
      a.recurrence_set = true;
    }
    else if (f == "--pipe-rr") a.opt.pipe_rr = std::stoi(need(i));
    else if (f == "--window") a.opt.form.window = tri(need(i), "--window");
    else if (f == "--carry") a.opt.form.carry = tri(need(i), "--carry");
    else if (f == "--interleave") a.opt.form.interleave = tri(need(i), "--interleave");
    else if (f == "--print-x") a.print_x = need(i);
    else if (f == "--report") a.report = need(i);
    else if (f == "--verify") a.verify = true;
    else if (f == "-h" || f == "--help") {
      std::fprintf(stderr, "flags: cuda_mpi_parallel_amd/cli_spec.py (shared with python -m cuda_mpi_parallel_amd)\n");
      std::exit(0);
    } else usage_error(f);
  }
  if (a.halo_transport == "rccl") a.opt.form.halo_pull = 0;  // no mapped peers: every ghost line exchanged
  if (!a.matrix.empty()) a.spec.kind = ProblemKind::Csr;
  if (a.spec.kind == ProblemKind::Csr) {
    if (a.matrix.empty()) usage_error("--problem csr needs --matrix FILE");
    a.mat.reset(read_matrix_market(a.matrix));
    if (!a.rhs_file.empty()) a.mat->set_rhs(read_vector(a.rhs_file));
    if (!a.rhs_set) a.spec.rhs = RhsKind::Reference;  // the file's b, ones without one
    a.rhs_set = true;
    a.spec.csr = &a.mat->view();
    a.spec.N = 0;
  }
  if (a.spec.kind == ProblemKind::RandomSPD) {
    if (a.spec.rows <= 0) a.spec.rows = 100000;
    if (a.spec.band <= 0) a.spec.band = 64;
    if (a.nnz_per_row > 0) a.spec.density = std::min(1.0, std::max(0.0, (a.nnz_per_row - 1.0) / (2.0 * a.spec.band)));
  }
  if (a.spec.kind != ProblemKind::Demo && !a.rhs_set) a.spec.rhs = RhsKind::Random;
  // generated problems default to the fast path (SELL-64/c8, falls back to d16 / plain SELL; the
  // single-reduction form); the built-in demo keeps the reference's CSR and two-reduction order
  if (a.spec.kind != ProblemKind::Demo && !a.format_set) a.opt.format = 3;
  if (a.spec.kind != ProblemKind::Demo && !a.recurrence_set) a.opt.recurrence = -1;
  // default grids, as make_problem(): 1024^2 (BASELINE config 1's size) and 128^3
  if (a.spec.kind == ProblemKind::Poisson2D && a.spec.N == 3) a.spec.N = 1024;
  if (a.spec.kind == ProblemKind::Poisson3D && a.spec.N == 3) a.spec.N = 128;
  return a;
}

class Barrier {
 public:
  explicit Barrier(int n) : n_(n) {}
  void wait() {
    std::unique_lock<std::mutex> lk(m_);
    if (failed_) fail("another rank failed");
    const int gen = gen_;
    if (++count_ == n_) { count_ = 0; ++gen_; cv_.notify_all(); return; }
    cv_.wait(lk, [&] { return gen != gen_ || failed_; });
    if (gen == gen_) fail("another rank failed");
  }
  void abort() {
    std::lock_guard<std::mutex> lk(m_);
    failed_ = true;
    cv_.notify_all();
  }
 private:
  std::mutex m_;
  std::condition_variable cv_;
  int n_, count_ = 0, gen_ = 0;
  bool failed_ = false;
};

struct RankOut {
  CgResult res;
  SolverInfo info;
  double true_rnorm = -1;
  double bench_seconds = 0;
  std::vector<double> x;
  int64_t row_begin = 0;
  std::string error, detail;
};

// Communicators of the ranks of this process: a rank that fails aborts them all, so the others
// leave their collectives with an error instead of waiting for it forever.
struct CommRegistry {
  std::mutex m;
  std::vector<Comm*> comms;
  bool failed = false;
  void add(Comm* c) {
    std::lock_guard<std::mutex> lk(m);
    comms.push_back(c);
    if (failed) c->abort();
  }
  void remove(Comm* c) {
    std::lock_guard<std::mutex> lk(m);
    comms.erase(std::remove(comms.begin(), comms.end(), c), comms.end());
  }
  void abort_all() {
    std::lock_guard<std::mutex> lk(m);
    failed = true;
    for (Comm* c : comms) c->abort();
  }
};
CommRegistry g_comms;

// Handle blobs of the rank threads (PeerHaloComm's local_handles / mailbox_handle), shared in memory:
// each thread deposits its own, a barrier, then every thread maps the others' (plain pointers).
struct Blobs {
  std::vector<std::string> halo, mailbox;
  explicit Blobs(int world) : halo(world), mailbox(world) {}
};

void run_rank(const Args& a, int rank, int world, const std::string& id_red, const std::string& id_halo,
              Barrier& bar, Blobs& blobs, const std::shared_ptr<LocalGroup>& group, bool want_x, RankOut& out) {
  try {
    if (hipSetDevice(group ? 0 : rank) != hipSuccess) fail("Device Set failed");  // CUDACG.cu:87-91
    std::shared_ptr<Comm> comm;
    std::shared_ptr<Communicator> inner;
    if (group) {
      inner = std::make_shared<LocalComm>(group, rank);  // --rehearse-ranks: the rank threads share GPU 0
    } else if (world > 1 || a.opt.force_comm) {
      comm.reset(a.comm_single ? new Comm(rank, world, unique_id_from_bytes(id_red))
                               : new Comm(rank, world, unique_id_from_bytes(id_red), unique_id_from_bytes(id_halo)));
      inner = comm;
    }
    if (comm) g_comms.add(comm.get());
    struct Unreg {
      Comm* c;
      ~Unreg() {
        if (c) g_comms.remove(c);
      }
    } unreg{comm.get()};
    struct AbortOnThrow {  // runs during unwinding, before `comm` is destroyed
      const std::shared_ptr<LocalGroup>* g;
      ~AbortOnThrow() {
        if (std::uncaught_exceptions() > 0) {
          g_comms.abort_all();
          if (*g) (*g)->abort();
        }
      }
    } guard{&group};
    // P > 1: the neighbours' halo buffers mapped (the in-kernel halo), every remaining exchange and, unless
    // the probe picks the IPC mailboxes, the all-reduce on the inner communicator
    std::shared_ptr<PeerHaloComm> peer;
    if (inner && world > 1 && a.halo_transport == "auto") {
      peer = std::make_shared<PeerHaloComm>(inner, rank, world);
      peer->set_halo_via_inner(true);
      // IPC all-reduce mailboxes: real GPUs only (rank threads sharing one GPU could queue one rank's
      // spinning all-reduce in front of another's pass)
      if (a.allreduce == "ipc" || (a.allreduce == "auto" && !group)) {
        const bool tolerant = a.allreduce == "auto";  // the probe's option: a rank that cannot map stays out
        try {
          blobs.mailbox[rank] = peer->mailbox_handle();
        } catch (const Error& e) {
          if (!tolerant) throw;
          std::fprintf(stderr, "[mcg] rank %d: IPC all-reduce mailbox unavailable (%s)\n", rank, e.what());
        }
        bar.wait();
        const bool all = std::all_of(blobs.mailbox.begin(), blobs.mailbox.end(), [](const std::string& b) { return !b.empty(); });
        try {
          if (!all) fail("ipc all-reduce: a rank could not export its mailbox");
          peer->attach_mailbox(blobs.mailbox);
        } catch (const Error& e) {
          if (!tolerant) throw;
          std::fprintf(stderr, "[mcg] rank %d: IPC all-reduce mailboxes not mapped (%s)\n", rank, e.what());
        }
        if (tolerant) peer->use_alt_allreduce(false);  // the transport probe decides
      }
    }
    Communicator* c = peer ? (Communicator*)peer.get() : inner.get();
    CgOptions opt = a.opt;
    if (a.fixed_iters > 0) { opt.tol = -1.0; opt.maxit = a.fixed_iters; }
    GpuCgSolver solver(a.spec, opt, rank, world, c);
    solver.setup();
    if (peer) {  // map the other threads' registered buffers; a rank that cannot stays unattached and the
                 // solver's check at the first reset turns the pull off on every rank
      blobs.halo[rank] = peer->local_handles();
      bar.wait();
      try {
        peer->attach(blobs.halo);
      } catch (const Error& e) {
        std::fprintf(stderr, "[mcg] rank %d: peer mapping failed (%s: %s); the halo stays on the inner communicator\n",
                     rank, e.what(), e.detail().c_str());
      }
    }
    out.info = solver.info();
    out.row_begin = solver.layout().row_begin;
    if (a.fixed_iters > 0) {
      solver.reset();
      out.info = solver.info();  // (the transport probe's choices)
      solver.run_iterations(a.warmup);
      solver.synchronize();
      bar.wait();
      const auto t0 = std::chrono::steady_clock::now();
      solver.run_iterations(a.fixed_iters);
      solver.synchronize();
      bar.wait();
      out.bench_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      solver.finalize();
      out.res = solver.result();
      out.res.solve_seconds = out.bench_seconds;
    } else if (!a.resume.empty()) {
      solver.load_checkpoint(a.resume);  // continue from the saved iteration
      out.res = solver.solve(true);
    } else {
      out.res = solver.solve();
    }
    if (a.verify) out.true_rnorm = solver.true_residual_norm();
    if (want_x) out.x = solver.x_local();
    out.info = solver.info();
  } catch (const Error& e) {
    out.error = e.what();
    out.detail = e.detail();
  } catch (const std::exception& e) {
    out.error = e.what();
  }
  if (!out.error.empty()) bar.abort();
}

}  // namespace

int main(int argc, char** argv) {
  Args a;
  try {
    a = parse(argc, argv);
  } catch (const Error& e) {
    std::printf("%s\n", e.what());
    return EXIT_FAILURE;
  } catch (const std::exception& e) {
    std::printf("invalid arguments: %s\n", e.what());
    return EXIT_FAILURE;
  }
  const int64_t n = global_rows(a.spec);
  const bool want_x = a.print_x == "yes" || (a.print_x == "auto" && n <= 1000);
  std::vector<double> x;
  CgResult res;
  SolverInfo info;
  double true_rnorm = -1;
  std::vector<size_t> rank_bytes;  // device bytes held by each rank's solver
  int world = a.cpu ? a.sim_ranks : a.gpus;

  try {
    if (a.cpu) {
      CgOptions opt = a.opt;
      if (a.fixed_iters > 0) { opt.tol = -1.0; opt.maxit = a.fixed_iters; }
      res = a.sim_ranks > 1 ? cpu_cg_partitioned(a.spec, a.sim_ranks, opt, &x) : cpu_cg(a.spec, opt, &x);
      info.n_global = n;
    } else {
      int ndev = 0;
      if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) fail("Device Set failed", "no HIP device");
      if (a.gpus < 1 || (a.gpus > ndev && !a.rehearse)) fail("Device Set failed", "requested more GPUs than present");
      std::string id_red, id_halo;
      if ((a.gpus > 1 || a.opt.force_comm) && !a.rehearse) {
        id_red = unique_id_bytes();
        id_halo = unique_id_bytes();
      }
      std::shared_ptr<LocalGroup> group;
      if (a.rehearse && a.gpus > 1) group = std::make_shared<LocalGroup>(a.gpus);
      Barrier bar(a.gpus);
      Blobs blobs(a.gpus);
      std::vector<RankOut> outs(a.gpus);
      std::vector<std::thread> ts;
      for (int r = 0; r < a.gpus; ++r)
        ts.emplace_back(run_rank, std::cref(a), r, a.gpus, std::cref(id_red), std::cref(id_halo), std::ref(bar),
                        std::ref(blobs), std::cref(group), want_x, std::ref(outs[r]));
      for (auto& t : ts) t.join();
      for (auto& o : outs)
        if (!o.error.empty()) fail(o.error, o.detail);
      res = outs[0].res;
      info = outs[0].info;
      true_rnorm = outs[0].true_rnorm;
      for (auto& o : outs) {
        rank_bytes.push_back(o.info.device_bytes);
        res.solve_seconds = std::max(res.solve_seconds, o.res.solve_seconds);
        res.setup_seconds = std::max(res.setup_seconds, o.res.setup_seconds);
      }
      if (want_x)
        for (auto& o : outs) x.insert(x.end(), o.x.begin(), o.x.end());
    }
  } catch (const Error& e) {
    std::printf("%s\n", e.what());
    if (!e.detail().empty()) std::fprintf(stderr, "[mcg] %s\n", e.detail().c_str());
    std::fflush(stdout);
    (void)hipDeviceReset();
    return EXIT_FAILURE;
  }

  if (want_x)
    for (double v : x) std::printf("%f\n", v);  // CUDACG.cu:361-364

  const double itps = res.iters_per_second();
  if (a.report == "json") {
    std::string per_rank = "[";
    for (size_t r = 0; r < rank_bytes.size(); ++r) per_rank += (r ? ", " : "") + std::to_string(rank_bytes[r]);
    per_rank += "]";
    // the P > 1 transports in effect and, if it ran, the transport probe's arms (mean us per iteration)
    char probe[512] = "null";
    if (info.probe_ran)
      std::snprintf(probe, sizeof probe,
                    "{\"pull_us\": %.3f, \"rccl_halo_us\": %.3f, \"ipc_ar_us\": %.3f, \"pull_bitwise\": %s, "
                    "\"ipc_ar_close\": %s, \"iters_timed\": %d, \"chosen\": \"%s+%s\"}",
                    info.probe_pull_us, info.probe_xchg_us, info.probe_alt_us, info.probe_pull_bitwise ? "true" : "false",
                    info.probe_alt_close ? "true" : "false", info.probe_iters, info.halo_pull ? "pull" : "exchange",
                    info.alt_allreduce ? "ipc" : "rccl");
    std::printf("{\"halo_pull\": %s, \"halo_transport\": \"%s\", \"allreduce\": \"%s\", \"transport_probe\": %s, "
                "\"rehearse_ranks\": %s, ",
                info.halo_pull ? "true" : "false",
                world < 2 || a.cpu ? "none" : info.halo_pull ? "in-kernel" : (a.rehearse ? "local" : "rccl"),
                world < 2 || a.cpu ? "none" : info.alt_allreduce ? "ipc" : (a.rehearse ? "local" : "rccl"), probe,
                a.rehearse ? "true" : "false");
    std::printf("\"problem\": \"%s\", \"n\": %lld, \"nnz_rank0\": %lld, \"ranks\": %d, \"device\": \"%s\", "
                "\"format\": \"%s\", \"iterations\": %d, \"converged\": %s, \"breakdown\": %s, \"rnorm\": %.6e, "
                "\"true_rnorm\": %.6e, \"setup_s\": %.6f, \"solve_s\": %.6f, \"it_per_s\": %.3f, "
                "\"device_bytes_rank0\": %zu, \"device_bytes_per_rank\": %s, \"rccl_version\": %d, "
                "\"rccl_library\": \"%s\"}\n",
                problem_name(a.spec).c_str(), (long long)n, (long long)info.nnz_local, world,
                a.cpu ? "cpu" : "gpu",
                a.cpu ? "csr"
                      : info.format == 5 ? "tiles" : info.format == 4 ? "sell64-aligned" : (info.format == 3 ? "sell64-c8"
                                          : (info.format == 2 ? "sell64-d16" : (info.format == 1 ? "sell64" : "csr"))),
                res.iterations,
                res.converged ? "true" : "false", res.breakdown ? "true" : "false", res.rnorm, true_rnorm,
                res.setup_seconds, res.solve_seconds, itps, info.device_bytes, per_rank.c_str(), rccl_version(),
                rccl_library().c_str());
  } else if (!want_x || n > 3) {
    std::fprintf(stderr,
                 "[mcg] problem=%s n=%lld ranks=%d iterations=%d converged=%d rnorm=%.3e solve=%.4fs "
                 "(%.2f it/s) setup=%.3fs\n",
                 problem_name(a.spec).c_str(), (long long)n, world, res.iterations, (int)res.converged, res.rnorm,
                 res.solve_seconds, itps, res.setup_seconds);
  }
  std::printf("Success\n");  // CUDACG.cu:365 CLEANUP("Success")
  return 0;
}
