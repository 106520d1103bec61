/*
 * ftar.h — C ABI of the MI355X-native FlexTree AllReduce (libftar.so).
 *
 * Plain pointers, sizes and enums only: no torch, no C++ types.  Every entry
 * point returns an ftar_status_t instead of exit()ing like the reference.
 * Device buffers are HBM pointers on the communicator's device; streams are
 * hipStream_t passed as void* so this header needs no HIP include.
 *
 * What each entry point replaces in the reference (DictXiong/AllReduce-Over-MPI):
 *
 *   ftar_reduce            FlexTree::reduce_sum<T> / reduce_band<T>
 *                            allreduce_over_mpi/mpi_mod.hpp:812-1031, :1034-1251
 *                          reduce_sum_gpu<T> + reduce_sum_1..20 kernels
 *                            vector_add/reduce_sum_gpu.h:4-316
 *   ftar_topo_parse        FlexTree::get_stages (FT_TOPO / FT_LONELY)
 *                            allreduce_over_mpi/mpi_mod.hpp:1419-1486
 *   ftar_topo_choose       cost_model getWidth + CostModel (argmin width list)
 *                            cost_model/GetWidth.h:42-47, cost_model/CostModel.h:82-120
 *   ftar_comm_init_rank    the MPI communicator the reference runs on (MPI_Comm_size/
 *                            rank, mpi_mod.hpp:781-809); transport = RCCL p2p
 *   ftar_allreduce         MPI_Allreduce_FT / static MPI_Allreduce
 *                            allreduce_over_mpi/mpi_mod.hpp:1723-1778
 *                          (ring_allreduce :1673-1719, tree_allreduce :1510-1671)
 *   ftar_schedule_json     Send/Recv_Operations + FMA_Send/Recv_Operations
 *                            allreduce_over_mpi/mpi_mod.hpp:258-766 (introspection)
 *
 * Results are bit-identical to the reference's CPU path for the same inputs
 * and FT_TOPO/FT_LONELY (same association order), see DESIGN.md §Parity.
 */
#ifndef FTAR_H
#define FTAR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FTAR_VERSION_MAJOR 0
#define FTAR_VERSION_MINOR 1
#define FTAR_MAX_STAGES 16
#define FTAR_MAX_K 64 /* max sources of one reduce (reference: 20, mpi_mod.hpp:811) */

typedef enum {
  FTAR_UINT8 = 0,   /* MPI_UINT8_T */
  FTAR_INT8 = 1,    /* MPI_INT8_T */
  FTAR_UINT16 = 2,  /* MPI_UINT16_T */
  FTAR_INT16 = 3,   /* MPI_INT16_T */
  FTAR_INT32 = 4,   /* MPI_INT32_T */
  FTAR_INT64 = 5,   /* MPI_INT64_T, MPI_LONG_LONG(_INT) */
  FTAR_FLOAT32 = 6, /* MPI_FLOAT */
  FTAR_FLOAT64 = 7, /* MPI_DOUBLE */
  FTAR_BOOL = 8,    /* MPI_C_BOOL: sum of bools == logical OR */
  FTAR_BFLOAT16 = 9 /* extension: fp32 accumulate, one RNE rounding per reduce */
} ftar_dtype_t;

typedef enum {
  FTAR_SUM = 0,  /* MPI_SUM */
  FTAR_BAND = 1  /* MPI_BAND (integer types only, as in the reference) */
} ftar_op_t;

typedef enum {
  FTAR_SUCCESS = 0,
  FTAR_ERR_INVALID_ARG = 1,
  FTAR_ERR_UNSUPPORTED = 2,   /* dtype/op pair the reference rejects too */
  FTAR_ERR_INVALID_TOPO = 3,  /* reference: "invalid FT_TOPO" + exit(1) */
  FTAR_ERR_HIP = 4,
  FTAR_ERR_RCCL = 5,
  FTAR_ERR_INTERNAL = 6,
  FTAR_ERR_TIMEOUT = 7,
  FTAR_ERR_NO_MEMORY = 8      /* a device allocation (scratch, staging, exchange buffer) failed */
} ftar_status_t;

/* Topology = FT_TOPO stage widths (bottom-up) + FT_LONELY count.  ring != 0
 * selects the ring schedule (reference: any width 1 in FT_TOPO). */
typedef struct {
  int nstages;
  int stages[FTAR_MAX_STAGES];
  int lonely;
  int ring;
} ftar_topo_t;

typedef struct ftar_comm* ftar_comm_t;
typedef struct {
  char internal[128];
} ftar_unique_id_t; /* == ncclUniqueId */

const char* ftar_version(void);
const char* ftar_status_string(ftar_status_t s);
/* Detail of the last failure on the calling thread ("" if none). */
const char* ftar_last_error(void);
size_t ftar_dtype_size(ftar_dtype_t dt);

/* ---- L3: k-way element-wise reduce on one device -------------------------
 * dst[i] = srcs[0][i] (+|&) srcs[1][i] (+|&) ... left to right, i < count.
 * srcs: HOST array of k device pointers; dst may alias srcs[0] (in place).
 * k == 1 copies (vector_add/reduce_sum.h:36-47).  stream: hipStream_t. */
ftar_status_t ftar_reduce(const void* const* srcs, int k, void* dst, size_t count, ftar_dtype_t dtype,
                          ftar_op_t op, void* stream);
/* Nested fold (extension; the one-round reduce-scatter of a multi-stage tree):
 * the k sources are the leaves, in depth-first order, of a mixed-radix tree
 * with bottom-up widths shape[0..nlevels) (product == k, nlevels <= 4).  Level
 * 0 folds shape[0] consecutive leaves, level 1 folds shape[1] consecutive
 * level-0 results, ... each node left to right; bf16 inner nodes are rounded
 * to bf16 (what a staged tree stores between its stages).  Integer sums and
 * AND are associative: the result equals ftar_reduce's.  nlevels <= 1 is
 * ftar_reduce. */
ftar_status_t ftar_reduce_nested(const void* const* srcs, int k, void* dst, size_t count, ftar_dtype_t dtype,
                                 ftar_op_t op, const int* shape, int nlevels, void* stream);

/* ---- topology ------------------------------------------------------------
 * ftar_topo_parse: FT_TOPO / FT_LONELY strings (NULL = unset) for nranks.
 * Unlike the reference (mpi_mod.hpp:1447-1475, which exit(1)s when FT_TOPO
 * is unset and P > 1), an unset FT_TOPO returns FTAR_ERR_INVALID_TOPO so the
 * caller can fall back to ftar_topo_choose. */
ftar_status_t ftar_topo_parse(const char* ft_topo, const char* ft_lonely, int nranks, ftar_topo_t* out);
/* FT_TOPO/FT_LONELY from the environment, else ftar_topo_choose(nranks, bytes). */
ftar_status_t ftar_topo_from_env(int nranks, size_t bytes, ftar_topo_t* out);
/* The topology the execution model (below) chooses among all ordered
 * factorizations of nranks (plus the ring) at the default data movement (the
 * one-round direct forms, the best piece): the reference's own question
 * (cost_model/CostModel.h:82-120).  FTAR_COST_MODEL=reference: the
 * reference's scores instead. */
ftar_status_t ftar_topo_choose(int nranks, size_t bytes, ftar_topo_t* out);
/* The candidate set the cost model scores, in the reference's getWidth order
 * (cost_model/GetWidth.h:42-47; its [1,P]/[P,1] entries = the ring), plus the
 * single-stage width-P tree right after the ring (getWidth omits it; FT_TOPO=P
 * is valid).  Writes up to max_out entries, returns the total count (<0 = error). */
int ftar_topo_candidates(int nranks, ftar_topo_t* out, int max_out);
/* Predicted seconds of one topology for a bucket of `bytes` at that default
 * data movement (direct forms, the model's piece). */
double ftar_topo_cost(const ftar_topo_t* topo, int nranks, size_t bytes);
/* Three of the execution model's constants (ftar_cost_set sets them all):
 * alpha = one p2p group's latency (us), link = one peer's one-direction
 * bandwidth (GB/s), hbm = the reduce kernel's rate (GB/s).  Process-wide; a
 * value <= 0 restores the default; the environment (FTAR_COST_ALPHA_US /
 * _LINK_GBPS / _HBM_GBPS) overrides both. */
ftar_status_t ftar_cost_set_params(double alpha_us, double link_gbps, double hbm_gbps);
ftar_status_t ftar_cost_get_params(double* alpha_us, double* link_gbps, double* hbm_gbps);

/* ---- execution model: (topology, data-movement form, pipeline piece) -------
 * The role of the reference's CostModel (cost_model/CostModel.h:82-120: a
 * width list chosen for a chunk size), re-derived for one MI355X node.  With
 * the one-round forms every topology moves tree(P)'s bytes, so what varies on
 * a node is the form and the piece size; the model prices both:
 *   per piece of a round: r(x) = max(alpha + x / link, issue)  (x = bytes per
 *   link), a fold of k sources (k + 1) * c / hbm on the reduce stream, the
 *   fill / drain of that two-stream pipeline simulated piece by piece; peer
 *   forms: barriers, xGMI loads / stores and their local copy pass.
 * Forms (ftar_comm_set_form; the env FTAR_FORM=auto|direct|stages|collective|
 * peer-read|peer-write at init): */
typedef enum {
  FTAR_FORM_AUTO = -1,       /* the model chooses per call (the default) */
  FTAR_FORM_DIRECT = 0,      /* one-round reduce-scatter + all-gather, RCCL p2p */
  FTAR_FORM_STAGES = 1,      /* the reference's rounds both ways, RCCL p2p */
  FTAR_FORM_COLLECTIVE = 2,  /* one-round reduce-scatter + ncclAllGather */
  FTAR_FORM_PEER_READ = 3,   /* IPC peer-direct read (FTAR_PEER_READ) */
  FTAR_FORM_PEER_WRITE = 4   /* IPC peer-direct write (FTAR_PEER_WRITE) */
} ftar_form_t;
/* The model's constants, SI-like units as named.  A field <= 0 in
 * ftar_cost_set restores its default; FTAR_COST_<FIELD> in the environment
 * (ALPHA_US, LINK_GBPS, HBM_GBPS, ISSUE_US, BARRIER_US, PEER_READ_GBPS,
 * PEER_WRITE_GBPS, COPY_GBPS, COLL_GBPS) overrides both.  peer_*_gbps and
 * coll_gbps default to 0 = unmeasured: those forms are then never chosen.
 * Process-wide; every rank must hold the same values (compared at a
 * communicator's first call). */
typedef struct {
  double alpha_us;        /* one p2p group (one piece of one round): launch + handshake */
  double link_gbps;       /* RCCL p2p, one peer, one direction */
  double hbm_gbps;        /* the fold's rate, algorithmic bytes ((k+1) x piece) per second */
  double issue_us;        /* host time to enqueue one piece of one round (groups, events, fold) */
  double barrier_us;      /* one stream-ordered barrier of the peer forms */
  double peer_read_gbps;  /* one peer, kernel loads over xGMI (0 = unmeasured) */
  double peer_write_gbps; /* one peer, kernel stores over xGMI (0 = unmeasured) */
  double copy_gbps;       /* local copy, algorithmic bytes (read + written) per second */
  double coll_gbps;       /* ncclAllGather: bytes each rank receives per second (0 = unmeasured) */
} ftar_cost_params_t;
ftar_status_t ftar_cost_set(const ftar_cost_params_t* params);
ftar_status_t ftar_cost_get(ftar_cost_params_t* params);
/* Calibration files: the constants a run on the node fitted (bench.py --save-cost), so every later
 * MPI_Allreduce_FT on that node prices with them.  One "<field> <value>" per line ('#' comments), the
 * fields named as in ftar_cost_params_t, values > 0; fields left out keep their defaults.  Precedence:
 * FTAR_COST_<FIELD> > ftar_cost_set > FTAR_COST_FILE's file > ftar_cost_load's file > the defaults.
 * FTAR_COST_FILE=<path> loads one (re-read when the variable changes; an unreadable or malformed file
 * leaves the constants as they were and fails communicator bring-up with FTAR_ERR_INVALID_ARG; unsetting
 * the variable drops its file's constants, not ftar_cost_load's).  ftar_cost_load(NULL) forgets the loaded
 * constants; a malformed file loads nothing.  ftar_cost_save writes the constants in effect. */
ftar_status_t ftar_cost_load(const char* path);
ftar_status_t ftar_cost_save(const char* path);
/* Predicted seconds of one AllReduce of `bytes` per rank: topology, form
 * (not AUTO), piece size (0 = whole blocks); registered != 0 prices the peer
 * forms on registered buffers (no local pass).  < 0: not runnable that way. */
double ftar_cost_predict(const ftar_topo_t* topo, int form, size_t chunk_bytes, int nranks, size_t bytes,
                         int registered);
typedef struct {
  ftar_topo_t topo;
  int form;            /* ftar_form_t */
  size_t chunk_bytes;  /* pipeline piece (the one-round and staged forms); 0 for the peer forms */
  double seconds;      /* predicted */
  int tied;            /* candidates priced equal to the choice (within 1e-9), the choice included:
                          1 = a strict argmin; > 1 = the model could not tell them apart */
  int tie_broken_by;   /* ftar_tie_t: the highest-ranked rule that set the choice apart from a tied one */
} ftar_exec_t;
/* Tie rules of ftar_exec_choose, in the order they apply. */
typedef enum {
  FTAR_TIE_NONE = 0,    /* no tie */
  FTAR_TIE_STAGES = 1,  /* the fewest stages (the ring last: the flat fold rounds bf16 once) */
  FTAR_TIE_FORM = 2,    /* the simpler form (ftar_form_t order) */
  FTAR_TIE_PIECE = 3    /* the larger piece (fewer p2p groups; whole blocks first) */
} ftar_tie_t;
#define FTAR_CHOOSE_TOPO 1  /* the topology is free (else inout->topo is used) */
#define FTAR_CHOOSE_FORM 2  /* the form is free (else inout->form) */
#define FTAR_CHOOSE_CHUNK 4 /* the piece size is free (else inout->chunk_bytes) */
#define FTAR_CHOOSE_PEER 8  /* the peer forms may be chosen (their rates permitting) */
/* The model's argmin over what `flags` leaves free; ties keep the fewest
 * stages, then the simpler form, then the larger piece, and the result says
 * how many candidates tied and which rule decided (tied, tie_broken_by): in
 * the direct form every one-round topology moves tree(P)'s bytes over the
 * same links, so those price alike and the stage count picks tree(P). */
ftar_status_t ftar_exec_choose(int nranks, size_t bytes, int flags, ftar_exec_t* inout);

/* The reference's own cost model, restated bit for bit
 * (cost_model/CostModel.h:1-120; tests/golden/costmodel.jsonl holds its
 * output).  ftar_topo_choose uses it instead of the xGMI model when
 * FTAR_COST_MODEL=reference (chunk = FTAR_COST_REF_CHUNK, default 100 as in
 * cost_model/main.cpp:23).
 *   ftar_cost_reference       score of one getWidth-style width list (a width
 *                             1 = the ring's [1,P]/[P,1]); < 0 where the
 *                             reference has no case (height 0 or > 9)
 *   ftar_topo_choose_reference its argmin over getWidth(P), first minimum wins
 *                             (CostModel.h:97); *index = position in that list
 *   ftar_cost_reference_candidates getWidth(P) (GetWidth.h:42-47) flattened:
 *                             returns the number of lists, their lengths in
 *                             lengths[], their widths concatenated in widths[] */
double ftar_cost_reference(const int* widths, int nwidths, int nranks, double chunk);
ftar_status_t ftar_topo_choose_reference(int nranks, double chunk, ftar_topo_t* out, int* index);
int ftar_cost_reference_candidates(int nranks, int* widths, int max_widths, int* lengths, int max_lists);
/* Writes "w0,w1,..+L" / "ring" into buf; returns needed length. */
int ftar_topo_format(const ftar_topo_t* topo, char* buf, size_t buflen);

/* ---- communicators -------------------------------------------------------- */
ftar_status_t ftar_get_unique_id(ftar_unique_id_t* id);
/* One process per GPU over RCCL p2p (xGMI). Collective across nranks. */
ftar_status_t ftar_comm_init_rank(ftar_comm_t* comm, int nranks, ftar_unique_id_t id, int rank, int device);
/* nranks communicators inside ONE process (thread transport: stream-ordered
 * device copies).  All ranks may share one device (test mode on a 1-GPU box).
 * Each ftar_allreduce on them must be issued from its own host thread, or via
 * ftar_allreduce_group. */
ftar_status_t ftar_comm_init_local(ftar_comm_t* comms, int nranks, const int* devices);
/* One process per rank, bootstrapped by the caller's own host collective (MPI,
 * gloo, ...): `allgather` copies `bytes` from `mine` into slot `rank` of `all`
 * on every rank and returns 0 on success.  Data moves only by the peer-direct
 * forms (IPC-mapped exchange or registered buffers; set FTAR_PEER_READ or
 * FTAR_PEER_WRITE): p2p transfers are FTAR_ERR_UNSUPPORTED, so staged and
 * lonely plans cannot run on it.  Barriers synchronize the stream and then
 * the host collective (blocking).  Ranks may share a device. */
typedef int (*ftar_host_allgather_fn)(const void* mine, void* all, size_t bytes, void* user);
ftar_status_t ftar_comm_init_host(ftar_comm_t* comm, int nranks, int rank, int device, ftar_host_allgather_fn allgather,
                                  void* user);
ftar_status_t ftar_comm_destroy(ftar_comm_t comm);
ftar_status_t ftar_comm_rank(ftar_comm_t comm, int* rank);
ftar_status_t ftar_comm_size(ftar_comm_t comm, int* size);
ftar_status_t ftar_comm_device(ftar_comm_t comm, int* device);
/* The communicator's transport: "rccl", "local" (in-process group) or "host" (ftar_comm_init_host). */
const char* ftar_comm_transport(ftar_comm_t comm);
/* Pipelining granularity of the transfers (bytes, rounded to 256 B); 0 = the
 * execution model's piece for each call (the default; FTAR_CHUNK_BYTES at
 * init fixes it).  get: 0 while the model chooses. */
ftar_status_t ftar_comm_set_chunk_bytes(ftar_comm_t comm, size_t bytes);
ftar_status_t ftar_comm_get_chunk_bytes(ftar_comm_t comm, size_t* bytes);
/* The data-movement form (ftar_form_t).  FTAR_FORM_AUTO (the default): the
 * execution model chooses per call among the forms the communicator can run
 * (peer forms only once their rates are set, ftar_cost_set); any other value
 * fixes it, as do ftar_comm_set_allgather / _reduce_scatter / _peer_direct
 * (get then reports the form those describe, or -2 for a mix no form names).
 * A host-bootstrapped communicator keeps its peer form.
 * ftar_comm_last_exec: what the last call on this communicator ran -- the
 * topology, the form of the path actually taken (host buffers on an RCCL
 * communicator run the pipelined p2p path whatever peer form is set; a ring
 * or host buffers replace the collective all-gather with the direct one; -2
 * for a mix no form names), the piece it ran in bytes (host buffers: the
 * host piece; 0: whole blocks, or a peer form on device buffers), and the
 * model's predicted seconds (-1: unpriced). */
ftar_status_t ftar_comm_set_form(ftar_comm_t comm, int form);
ftar_status_t ftar_comm_get_form(ftar_comm_t comm, int* form);
ftar_status_t ftar_comm_last_exec(ftar_comm_t comm, ftar_exec_t* out);
/* How the all-gather phase is moved.  After the reduce-scatter stages every
 * rank holds exactly one fully reduced block (block r on trees, lonely ranks
 * included; block (r+1) mod P on the ring), so the phase only delivers final
 * values and every form gives bit-identical results:
 *   FTAR_AG_STAGES      the reference's rounds (ring: P-1 neighbour steps,
 *                       tree: the k stages reversed, mpi_mod.hpp:1620-1644, :1705-1715)
 *   FTAR_AG_DIRECT      one p2p group: each rank sends its block to all P-1
 *                       peers at once (every xGMI link busy; default)
 *   FTAR_AG_COLLECTIVE  one ncclAllGather (non-lonely trees with P | count;
 *                       otherwise DIRECT)
 * Default: FTAR_ALLGATHER=stages|direct|collective at init, else DIRECT. */
typedef enum { FTAR_AG_STAGES = 0, FTAR_AG_COLLECTIVE = 1, FTAR_AG_DIRECT = 2 } ftar_allgather_t;
ftar_status_t ftar_comm_set_allgather(ftar_comm_t comm, ftar_allgather_t mode);
ftar_status_t ftar_comm_get_allgather(ftar_comm_t comm, ftar_allgather_t* mode);
/* How the ring's reduce-scatter is moved.  The ring folds block b as
 * x_b + x_{b+1} + ... + x_{b+P-1} (left to right, indices mod P; the reference's
 * own+recv per hop is that fold since IEEE addition commutes), finishing on rank
 * b-1 (mpi_mod.hpp:1689-1703):
 *   FTAR_RS_STAGES  the reference's P-1 neighbour steps (one xGMI link per rank)
 *   FTAR_RS_DIRECT  rank b-1 gathers every rank's block b in ONE round over all
 *                   links and folds them in that order with one k=P reduce
 *                   (bf16: rounded after every add, i.e. once per hop, as staged)
 * Identical results.  Multi-stage trees without lonely ranks (at most 4
 * stages) likewise: FTAR_RS_DIRECT gathers the P copies of block r on rank r
 * in one round and folds them as the tree would (ftar_reduce_nested), bit for
 * bit; lonely layouts and single-stage trees keep their stages.
 * Default: FTAR_REDUCE_SCATTER=stages|direct, else DIRECT. */
typedef enum { FTAR_RS_STAGES = 0, FTAR_RS_DIRECT = 1 } ftar_reduce_scatter_t;
ftar_status_t ftar_comm_set_reduce_scatter(ftar_comm_t comm, ftar_reduce_scatter_t mode);
ftar_status_t ftar_comm_get_reduce_scatter(ftar_comm_t comm, ftar_reduce_scatter_t* mode);

/* Peer-direct data movement (extension; default off, FTAR_PEER_DIRECT=1|read
 * or 2|write at init).  For one-round plans (the ring, and trees without
 * lonely ranks, under FTAR_RS_DIRECT-or-single-stage + FTAR_AG_DIRECT), the
 * blocks move by kernel loads/stores through IPC-mapped, comm-owned exchange
 * buffers over xGMI instead of RCCL p2p into scratch:
 *   FTAR_PEER_READ   each rank's fold reads the other ranks' copies of its
 *                    block from their exchange buffers, and the all-gather
 *                    pulls every final block (three stream-ordered barriers);
 *   FTAR_PEER_WRITE  each rank pushes its copy of every peer's block into that
 *                    peer's buffer, folds locally, and pushes its final block
 *                    to every peer (three barriers: the last keeps
 *                    my exchange buffer until my copy-out has read it).
 * The plan's fold is executed unchanged: same bits.  Other plans keep RCCL p2p. */
typedef enum { FTAR_PEER_OFF = 0, FTAR_PEER_READ = 1, FTAR_PEER_WRITE = 2 } ftar_peer_mode_t;
ftar_status_t ftar_comm_set_peer_direct(ftar_comm_t comm, int mode);
ftar_status_t ftar_comm_get_peer_direct(ftar_comm_t comm, int* mode);
/* Registered (symmetric) buffers for the peer forms, like RCCL's user-buffer
 * registration.  Collective: every rank registers its own buffer of the same
 * role in the same call order; *reg is the same id on every rank.  A call
 * whose buffers lie in registrations -- on EVERY rank, at the SAME offsets
 * -- skips the peer forms' local pass: READ (sendbuf and recvbuf registered)
 * reads the peers' inputs and final blocks in place, three barriers, no
 * copy; WRITE (recvbuf registered) pushes final blocks straight into the
 * peers' outputs, two barriers, no copy.  Mixing registered and unregistered
 * buffers across ranks in one call is undefined.  deregister is local; the
 * buffer must not be freed before it (or before the calls using it ended).
 * The buffer must not be written while it is being registered: every peer
 * verifies its mapping against the owner's current first 16 bytes.
 * Under HIP runtimes older than 7.2 an allocation whose size has bit 31 set
 * cannot be registered (FTAR_ERR_HIP on every rank): those runtimes block in
 * hipIpcOpenMemHandle for such sizes.  FTAR_IPC_SIZE_GUARD=0|1 overrides. */
ftar_status_t ftar_comm_register(ftar_comm_t comm, void* buf, size_t bytes, int* reg);
ftar_status_t ftar_comm_deregister(ftar_comm_t comm, int reg);

/* ---- AllReduce (device resident) -------------------------------------------
 * sendbuf == NULL or == recvbuf: in place (MPI_IN_PLACE).  topo == NULL:
 * FT_TOPO/FT_LONELY read from the environment at THIS call, as get_stages is
 * on every MPI_Allreduce_FT call (mpi_mod.hpp:1732); both unset: the cost
 * model's choice; set but invalid for the communicator's size:
 * FTAR_ERR_INVALID_TOPO before anything is enqueued (the reference exit(1)s,
 * :1471-1475), 1-rank communicators included.  Enqueued on `stream`; returns
 * once enqueued. */
ftar_status_t ftar_allreduce(const void* sendbuf, void* recvbuf, size_t count, ftar_dtype_t dtype, ftar_op_t op,
                             const ftar_topo_t* topo, ftar_comm_t comm, void* stream);
/* Drive every rank of an ftar_comm_init_local group from this one call
 * (pooled host threads, one per rank at once); returns once every rank's
 * work is enqueued on its stream (streams == NULL: each device's NULL
 * stream), like ftar_allreduce -- synchronize the streams before reading
 * the results from the host.  ftar_allreduce_host_group returns once the
 * host buffers hold the result.
 * Under stream capture pass the capture stream itself for every rank (the
 * call is then captured serially, one graph chain); streams forked per rank
 * from the capture are refused with FTAR_ERR_UNSUPPORTED, as HIP's
 * hipStreamEndCapture recurses without end on them. */
ftar_status_t ftar_allreduce_group(const void* const* sendbufs, void* const* recvbufs, size_t count,
                                   ftar_dtype_t dtype, ftar_op_t op, const ftar_topo_t* topo, ftar_comm_t* comms,
                                   int nranks, void* const* streams);

/* ---- AllReduce of HOST buffers (the reference's own setting) ---------------
 * Replaces MPI_Allreduce_FT's host-memory contract (mpi_mod.hpp:1723-1778).
 * sendbuf/recvbuf are host memory (sendbuf == NULL or == recvbuf: in place);
 * page-lock them (hipHostRegister / hipHostMalloc) or the copies are not
 * asynchronous.  The bucket moves through a grow-only device staging buffer in
 * pieces of host_chunk_bytes per block: H2D of later pieces, the exchange and
 * reduce of the current ones, and D2H of finished ones run at once (stage s+1
 * trails stage s by one piece), so PCIe in and out overlap.  Same blocks,
 * same fold order, same bits as ftar_allreduce.  Enqueued on `stream`; the
 * host buffers must stay untouched until it completes. */
ftar_status_t ftar_allreduce_host(const void* sendbuf, void* recvbuf, size_t count, ftar_dtype_t dtype,
                                  ftar_op_t op, const ftar_topo_t* topo, ftar_comm_t comm, void* stream);
ftar_status_t ftar_allreduce_host_group(const void* const* sendbufs, void* const* recvbufs, size_t count,
                                        ftar_dtype_t dtype, ftar_op_t op, const ftar_topo_t* topo,
                                        ftar_comm_t* comms, int nranks, void* const* streams);
/* Co-scheduling of the fold with the transport: the reduce stream runs on
 * `cus` of the device's CUs (spread evenly; 0 = all, the default), so the
 * comm stream's kernels (RCCL p2p, copies) always find free CUs while a
 * piece's fold runs (FTAR_REDUCE_CUS at init).  Same bits either way.
 * In-process (local) and host-bootstrapped communicators only: on an RCCL
 * communicator any cus other than 0 returns FTAR_ERR_UNSUPPORTED, and
 * FTAR_REDUCE_CUS fails ftar_comm_init_rank the same way.  The CU-masked
 * stream is a blocking stream on a hardware queue of its own, and over RCCL
 * two stress runs stalled ranks with it. */
ftar_status_t ftar_comm_set_reduce_cus(ftar_comm_t comm, int cus);
ftar_status_t ftar_comm_get_reduce_cus(ftar_comm_t comm, int* cus);
/* Host-mode piece size per block (bytes, rounded to 256 B); 0 = auto: 16 MiB,
 * at least 1/64 of a block (FTAR_HOST_CHUNK_BYTES at init). */
ftar_status_t ftar_comm_set_host_chunk_bytes(ftar_comm_t comm, size_t bytes);
ftar_status_t ftar_comm_get_host_chunk_bytes(ftar_comm_t comm, size_t* bytes);

/* ---- diagnostics ---------------------------------------------------------------
 * RCCL's own ncclAllReduce on the communicator's RCCL comm (ring/tree of the
 * vendor library, reduction inside RCCL): the yardstick bench.py reports next
 * to ftar at N > 1.  FTAR_ERR_UNSUPPORTED on local (in-process) groups. */
ftar_status_t ftar_rccl_allreduce(const void* sendbuf, void* recvbuf, size_t count, ftar_dtype_t dtype, ftar_op_t op,
                                  ftar_comm_t comm, void* stream);
/* xGMI calibration (collective; every rank calls it): GB/s seen by this rank
 * for copy kernels through the peer-direct exchange buffers, all ranks running
 * the same pattern at once -- gbps[0] local HBM copy, [1] read from one peer
 * (ring neighbour), [2] read from all peers at once (aggregate), [3] write to
 * one peer, [4] write to all peers at once (aggregate), all by copy kernels;
 * [5] read from / [6] write to all peers by the DMA engines (one
 * hipMemcpyAsync per peer, each on its own stream).  bytes_per_peer per
 * copy, `iters` timed launches; grows the exchange buffer to 2*P*bytes. */
ftar_status_t ftar_xgmi_probe(ftar_comm_t comm, size_t bytes_per_peer, int iters, double* gbps, int n);
/* Phase timing of the last call on this communicator (diagnostic; off by
 * default): timing events at the phase boundaries -- per stage "moved" (comm
 * stream) and "reduced" (reduce stream) for the p2p executor in device mode,
 * every copy/fold/barrier for the peer forms.  ftar_comm_phase_json waits for
 * them and writes [["start", 0.0], [name, ms since start], ...]; returns the
 * needed length or < 0 on error. */
ftar_status_t ftar_comm_set_phase_timing(ftar_comm_t comm, int enable);
long ftar_comm_phase_json(ftar_comm_t comm, char* buf, size_t buflen);

/* ---- introspection (tests) -------------------------------------------------
 * FMA-level schedule of `rank` (same JSON shape as the reference dump in
 * tests/golden/schedules.jsonl). Returns needed length, or <0 on error. */
long ftar_schedule_json(const ftar_topo_t* topo, int nranks, int rank, size_t count, char* buf, size_t buflen);
/* Executable plan of `rank` (JSON): stages of transfers/reduces, scratch size,
 * and the forms actually used. */
long ftar_plan_json(const ftar_topo_t* topo, int nranks, int rank, size_t count, ftar_allgather_t allgather,
                    ftar_reduce_scatter_t reduce_scatter, char* buf, size_t buflen);

#ifdef __cplusplus
}
#endif
#endif /* FTAR_H */
