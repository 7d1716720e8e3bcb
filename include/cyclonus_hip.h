/* cyclonus_hip.h — C ABI of libcyclonus_hip.so, the MI355X (gfx950) NetworkPolicy verdict engine.
 *
 * Drop-in boundary for the simulated-connectivity path of cyclonus (reference paths are
 * relative to the reference repository, github.com/mattfenwick/cyclonus @ johnSchnake fork):
 *
 *   cyc_policy_build_json   replaces matcher.BuildNetworkPolicies(simplify, netpols)
 *                           pkg/matcher/builder.go:11-26 (+ Policy.Simplify policy.go:176-183)
 *   cyc_policy_load_ir_json accepts json.Marshal(*matcher.Policy) — the already-built Go policy
 *                           a cgo binding holds in SimulatedJobRunner.Policies (jobrunner.go:64-66)
 *   cyc_resources_load_json probe.Resources (pkg/connectivity/probe/resources.go:15-19) as JSON
 *   cyc_probe_prepare       Resources.GetJobsForProbeConfig (resources.go:274-364) for a batch of
 *                           generator.ProbeConfig values (PortProtocol | AllAvailable)
 *   cyc_probe_run           Runner.RunProbeForConfig (jobrunner.go:29-58) -> SimulatedJobRunner.RunJobs
 *                           (jobrunner.go:68-94) -> Policy.IsTrafficAllowed (policy.go:131-174) for
 *                           every (src pod, dst pod, job) cell, as packed bit-planes
 *   cyc_query_traffic       Policy.IsTrafficAllowed for arbitrary matcher.Traffic values, including
 *                           external peers (analyze.go:209-225 query-traffic)
 *
 * Conventions: every function returns a cyc_status; on failure cyc_last_error(ctx) holds the
 * message (for CYC_ERR_PANIC_* it is the text of the Go panic the reference would raise).
 * Inputs are copied during the call (no caller pointer is retained, cgo-safe).  A context is
 * not internally locked: use one per thread.  Plane layout (W = ceil(P/64) 64-bit words):
 *   status[d*K + k]                      cyc_job_status of destination pod d, job slot k
 *   ingress[((d-row_lo)*K + k)*W + s/64]  bit s%64: ingress verdict of s -> d, slot k
 *   egress [((s-row_lo)*K + k)*W + d/64]  bit d%64: egress verdict of s -> d, slot k
 * i.e. each plane is keyed by the pod the direction's policies TARGET (ingress: destination,
 * egress: source; policy.go:143-149).  Combined = ingress AND egress (policy.go:123-125).
 * Bits of non-VALID slots are 0; their Ingress/Egress/Combined follow jobrunner.go:36-55.
 */
#ifndef CYCLONUS_HIP_H
#define CYCLONUS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  CYC_OK = 0,
  CYC_ERR_ARG = 1,             /* bad argument / call order */
  CYC_ERR_JSON = 2,            /* malformed input document */
  CYC_ERR_INVALID_POLICY = 3,  /* builder.go:39,174-181 panics */
  CYC_ERR_PANIC_IP = 4,        /* ippeermatcher.go:46-48 panic: unparsable pod IP */
  CYC_ERR_PANIC_CIDR = 5,      /* ippeermatcher.go:46-48 panic: unparsable CIDR / except */
  CYC_ERR_PANIC_SELECTOR = 6,  /* labelselector.go:57 panic("invalid operator") */
  CYC_ERR_DUPLICATE_KEY = 7,   /* table.go:45 via utils.DoOrDie (log.Fatalf) */
  CYC_ERR_HIP = 8,
  CYC_ERR_OOM = 9,
  CYC_ERR_RCCL = 10,
  CYC_ERR_PANIC_RUNTIME = 11   /* Go runtime panic in the job expansion: a pod without containers is a
                                  job's podFrom (resources.go:296,349, Containers[0]) */
} cyc_status;

typedef enum {
  CYC_JOB_NONE = 0,               /* no job in this slot (AllAvailable, fewer containers) */
  CYC_JOB_VALID = 1,              /* Ingress/Egress from the planes */
  CYC_JOB_BAD_NAMED_PORT = 2,     /* Ingress=invalidnamedport, Egress=unknown (jobrunner.go:47-55) */
  CYC_JOB_BAD_PORT_PROTOCOL = 3   /* Ingress=invalidportprotocol, Egress=unknown (:36-45) */
} cyc_job_status;

typedef struct cyc_ctx cyc_ctx;

typedef struct {
  int64_t pods;        /* P */
  int64_t slots;       /* K: job slots per destination pod over all probe configs */
  int64_t words;       /* W = ceil(P/64) */
  int64_t configs;     /* number of probe configs */
  int64_t targets_in;  /* ingress targets after merge/simplify */
  int64_t targets_eg;
  int64_t peers;
  int64_t classes_in;  /* filled after cyc_probe_run */
  int64_t classes_eg;
  int64_t may_panic;   /* 1 if evaluation can reach a Go panic (invalid CIDR/IP/operator) */
  int64_t selectors;   /* S: distinct label selectors */
  int64_t label_sets;  /* L: distinct pod / namespace label sets */
  int64_t pod_peers;   /* pod-selector peers (pod, namespace or both) */
  int64_t ip_peers;    /* IPBlock peers */
  int64_t descriptors; /* D: distinct job descriptors (port, port name, protocol) */
  int64_t max_word_runs; /* most egress-identity runs in one 64-pod word */
} cyc_probe_shape;

/* ABI revision of this header: bumped whenever a struct's layout or a field's meaning changes.  A
 * binding checks cyc_abi_version() == CYC_ABI_VERSION once at start-up so a library and a binding
 * built against different headers fail loudly instead of misreading each other's structs. */
#define CYC_ABI_VERSION 2

/* context / errors */
int cyc_abi_version(void);
int cyc_ctx_create(int device_id, cyc_ctx** out);
void cyc_ctx_destroy(cyc_ctx* ctx);
const char* cyc_last_error(const cyc_ctx* ctx);
const char* cyc_version(void);

/* policy compile: JSON array (or List / single object) of networking.k8s.io/v1 NetworkPolicy */
int cyc_policy_build_json(cyc_ctx* ctx, int simplify, const char* netpols_json, size_t len);
/* policy load: json.Marshal(*matcher.Policy) produced by the Go reference */
int cyc_policy_load_ir_json(cyc_ctx* ctx, const char* policy_json, size_t len);
/* export the compiled policy as json.Marshal(*matcher.Policy) would; returns bytes needed (+1) and
 * writes the NUL-terminated text when cap holds it (a smaller cap writes nothing); returns
 * -(cyc_status) on failure (no policy loaded, or the dump failed) with cyc_last_error set */
int64_t cyc_policy_ir_json(cyc_ctx* ctx, char* buf, size_t cap);

/* probe model: probe.Resources JSON ({"Namespaces": {...}, "Pods": [...]}) */
int cyc_resources_load_json(cyc_ctx* ctx, const char* resources_json, size_t len);

/* probe configs: JSON array of {"Port": <int|string>, "Protocol": "TCP"} or {"AllAvailable": true};
 * flattens + uploads all tables and allocates device scratch.  Fills *shape. */
int cyc_probe_prepare(cyc_ctx* ctx, const char* probes_json, size_t len, cyc_probe_shape* shape);

/* ---- Flat-table ingestion (no JSON): what a cgo binding passes straight from its Go values.
 * Every string is an index into one string table (duplicates allowed); maps and lists are
 * [n + 1] offset arrays into shared element arrays; optional arrays may be NULL.  The caller keeps
 * ownership: everything is copied during the call (cgo rule: no Go pointer is retained).  Indices
 * and offsets are validated (CYC_ERR_ARG names the first bad one). */
typedef struct {
  int64_t n;           /* strings */
  const char* bytes;   /* their bytes, concatenated (Go strings: any bytes, NUL included) */
  const int64_t* off;  /* [n + 1]: string i = bytes[off[i], off[i + 1]) */
} cyc_strings;

/* probe.Resources (pkg/connectivity/probe/resources.go:15-19, pod.go:44-51,173-179) */
typedef struct {
  cyc_strings str;
  /* Namespaces map[string]map[string]string */
  int64_t n_namespaces;
  const int32_t* ns_name;        /* [n_namespaces] the map key */
  const uint8_t* ns_nil;         /* [n_namespaces] 1: a nil label map (optional) */
  const int64_t* ns_label_off;   /* [n_namespaces + 1] into ns_label_key / ns_label_val */
  const int32_t *ns_label_key, *ns_label_val;
  /* Pods []*Pod, in order */
  int64_t n_pods;
  const int32_t *pod_ns, *pod_name, *pod_ip;  /* [n_pods] Namespace, Name, IP */
  const int64_t* pod_label_off;  /* [n_pods + 1] into label_key / label_val (Labels map) */
  const int32_t *label_key, *label_val;
  const int64_t* pod_cont_off;   /* [n_pods + 1] into the container arrays (Containers) */
  const int32_t *cont_name, *cont_port, *cont_proto, *cont_port_name;  /* Name, Port, Protocol, PortName */
  const uint8_t* pod_nil;        /* [n_pods] optional: bit 0 Labels == nil, bit 1 Containers == nil
                                    (json.Marshal fidelity only: cyc_resources_json writes null) */
} cyc_resource_tables;

/* generator.ProbeConfig (pkg/generator/probeconfig.go): AllAvailable, or PortProtocol{Port intstr, Protocol} */
typedef struct {
  int32_t all_available;  /* 1: one job per destination container (resources.go:336-364) */
  int32_t port_is_name;   /* intstr.Type: 0 Int (port), 1 String (port_name) */
  int32_t port;
  /* Go strings as (pointer, byte length): any bytes, NUL included; NULL with length 0 = "".
   * (ABI 2 renamed the pointers from port_name / protocol when the lengths were added, so a caller
   * written against ABI 1 that set only the pointer no longer compiles.) */
  const char* port_name_ptr;  /* the named port */
  int64_t port_name_len;
  const char* protocol_ptr;   /* the raw protocol string (compared as is: "tcp" != "TCP") */
  int64_t protocol_len;
} cyc_probe_config;

/* *matcher.Policy after BuildNetworkPolicies (+ Simplify) (pkg/matcher/policy.go:11-14,
 * target.go:11-23, peermatcher.go, podpeermatcher.go, ippeermatcher.go, portmatcher.go): the already
 * built Go policy, flattened.  Targets are given per direction (ingress then egress); each holds its
 * ordered peer list; a peer's port matcher is an index (peers of one rule may share one). */
typedef enum { CYC_PEER_ALL = 0, CYC_PEER_PORTS = 1, CYC_PEER_POD = 2, CYC_PEER_IP = 3 } cyc_peer_kind;
typedef enum { CYC_NS_EXACT = 0, CYC_NS_ALL = 1, CYC_NS_LABEL = 2 } cyc_ns_kind;
typedef enum { CYC_PORT_ANY = 0, CYC_PORT_NUMBER = 1, CYC_PORT_NAME = 2 } cyc_port_kind;
typedef struct {
  cyc_strings str;
  /* metav1.LabelSelector: MatchLabels, then MatchExpressions {Key, Operator, Values} */
  int64_t n_selectors;
  const int64_t* sel_label_off;  /* [n_selectors + 1] into sel_label_key / sel_label_val */
  const int32_t *sel_label_key, *sel_label_val;
  const int64_t* sel_expr_off;   /* [n_selectors + 1] into expr_key / expr_op / expr_value_off */
  const int32_t *expr_key, *expr_op;  /* expr_op: the operator text ("In", "NotIn", "Exists", "DoesNotExist";
                                         anything else panics when reached, labelselector.go:57) */
  const int64_t* expr_value_off; /* [n_exprs + 1] into expr_value */
  const int32_t* expr_value;
  /* PortMatcher: AllPortMatcher, or SpecificPortMatcher{Ports, PortRanges} */
  int64_t n_port_matchers;
  const uint8_t* pm_all;         /* [n_port_matchers] 1: AllPortMatcher */
  const uint8_t *pm_ports_nil, *pm_ranges_nil;  /* optional: nil slices (json.Marshal fidelity only) */
  const int64_t* pm_port_off;    /* [n_port_matchers + 1] into port_* (PortProtocolMatcher) */
  const uint8_t* port_kind;      /* cyc_port_kind: Port == nil / number / name */
  const int32_t* port_value;     /* the number, or the name's string index */
  const int32_t* port_proto;     /* Protocol string index */
  const int64_t* pm_range_off;   /* [n_port_matchers + 1] into range_* (PortRangeMatcher) */
  const int32_t *range_from, *range_to, *range_proto;
  /* targets: n_targets[0] ingress, then n_targets[1] egress, each direction sorted or not (the
   * library orders them by primary key, target.go:57-62, as Go's map keys) */
  int64_t n_targets[2];
  const int32_t* target_ns;      /* Namespace string index */
  const int32_t* target_sel;     /* PodSelector: selector index */
  const uint8_t* target_peers_nil; /* optional: Peers == nil (json.Marshal fidelity only) */
  const int64_t* target_peer_off;  /* [n_in + n_eg + 1] into peer_* (ordered: Target.Allows short-circuits) */
  const int64_t* target_rule_off;  /* optional [n_in + n_eg + 1] into rule_name (SourceRules' names) */
  const int32_t* rule_name;
  /* peers */
  const uint8_t* peer_kind;      /* cyc_peer_kind */
  const int32_t* peer_port;      /* port matcher index (ignored for CYC_PEER_ALL) */
  const uint8_t* peer_ns_kind;   /* cyc_ns_kind (pod peers) */
  const int32_t* peer_ns;        /* CYC_NS_EXACT: namespace string index; CYC_NS_LABEL: selector index */
  const int32_t* peer_pod_sel;   /* pod peers: selector index, -1 = all pods */
  const int32_t* peer_cidr;      /* IP peers: CIDR string index */
  const int64_t* peer_except_off;  /* [n_peers + 1] into except_cidr (IP peers' Except) */
  const uint8_t* peer_except_nil;  /* optional: Except == nil (json.Marshal fidelity only) */
  const int32_t* except_cidr;
} cyc_policy_tables;

/* the flat counterparts of cyc_resources_load_json, cyc_policy_load_ir_json and cyc_probe_prepare */
int cyc_resources_load(cyc_ctx* ctx, const cyc_resource_tables* tables);
int cyc_policy_load(cyc_ctx* ctx, const cyc_policy_tables* tables);
int cyc_probe_prepare_configs(cyc_ctx* ctx, const cyc_probe_config* configs, int64_t n, cyc_probe_shape* shape);
/* the loaded probe model as json.Marshal(*probe.Resources) would write it (Pod.ServiceIP and
 * Container.BatchJobs are not kept; nil label maps and container slices as null: from JSON input an
 * absent or null field, from flat tables ns_nil / pod_nil); returns bytes needed (+1) or
 * -(cyc_status), as cyc_policy_ir_json */
int64_t cyc_resources_json(cyc_ctx* ctx, char* buf, size_t cap);

/* Compute the verdict planes on the GPU for target-pod rows [row_lo, row_hi) (rows are pods in
 * Resources.Pods order; pass 0, P for the whole table).  Device pointers; `hip_stream` is the
 * hipStream_t to enqueue on (NULL = the HIP default stream, as with every HIP API).  Asynchronous
 * unless the inputs can panic (then it synchronises to report the first panicking job in job
 * order, as the reference would).  The planes must be device memory (hipMalloc and the like), read
 * back by hipMemcpy or by kernels after the stream: the run's events release at device scope, so
 * host-mapped, non-coherent memory is not made visible to the host by a stream synchronisation. */
int cyc_probe_run(cyc_ctx* ctx, void* hip_stream, uint64_t* d_ingress, uint64_t* d_egress, uint8_t* d_status,
                  int64_t row_lo, int64_t row_hi);

/* Same, into host buffers (allocates + copies; synchronous). */
int cyc_probe_run_host(cyc_ctx* ctx, uint64_t* ingress, uint64_t* egress, uint8_t* status, int64_t row_lo,
                       int64_t row_hi);

/* ---- Row partitions for one-process-per-GPU runs (north_star: "source-pod rows shard across the
 * GPUs").  A rank runs rows [row_lo, row_hi) of the pods under one of two partitions:
 *   CYC_ROWS_TARGET  the rows are TARGET pods of both planes (cyc_probe_run's layout above): rank r
 *                    holds the ingress rows of destinations and the egress rows of sources in the range.
 *   CYC_ROWS_SOURCE  the rows are SOURCE pods: rank r holds every cell (s in [row_lo, row_hi), d, k),
 *                    i.e. Table.Get(from, *) for its sources (pkg/connectivity/probe/table.go:54-56, the
 *                    reference's jobs are generated source-major, resources.go:286-287):
 *                      egress [((s - row_lo)*K + k)*W  + d/64]              bit d%64 (full rows of its sources)
 *                      ingress[(d*K + k)*Wr + (s/64 - row_lo/64)]          bit s%64, for EVERY destination d,
 *                    Wr = ceil(row_hi/64) - row_lo/64 words: the rank's slice of each ingress row.
 *                    row_lo must be a multiple of 64, and row_hi too unless it is P, so the slices of
 *                    a partition tile every ingress row.  The rank's peer rows and ingress class rows
 *                    cover only its words, so its front work shrinks with the partition too.
 * The union of the ranks' planes is the whole table either way, with no data exchange (the inputs are
 * replicated); assembling it on every rank is one all-gather per plane (cyclonus_amd/shard.py). */
typedef enum { CYC_ROWS_TARGET = 0, CYC_ROWS_SOURCE = 1 } cyc_rows;

/* Plane shapes of rows [row_lo, row_hi) under `partition`: out[0] ingress rows, out[1] words per
 * ingress (row, slot), out[2] egress rows, out[3] words per egress (row, slot), out[4] the ingress
 * window's first word (0 for target rows).  Needs cyc_probe_prepare. */
int cyc_rows_layout(cyc_ctx* ctx, int partition, int64_t row_lo, int64_t row_hi, int64_t* out, int n);
int cyc_probe_run_rows(cyc_ctx* ctx, void* hip_stream, uint64_t* d_ingress, uint64_t* d_egress, uint8_t* d_status,
                       int partition, int64_t row_lo, int64_t row_hi);
int cyc_probe_run_host_rows(cyc_ctx* ctx, uint64_t* ingress, uint64_t* egress, uint8_t* status, int partition,
                            int64_t row_lo, int64_t row_hi);

/* ---- Device-resident verdict tables: the lazy probe.Table (pkg/connectivity/probe/table.go:24-56).
 * The reference's Runner.RunProbeForConfig returns *Table = NewTableFromJobResults(resources,
 * runProbe(jobs)) (jobrunner.go:29-58, table.go:38-48): one Item per (from, to) pod pair holding a
 * JobResult {Ingress, Egress, Combined} per job key.  A cyc_table keeps the packed planes on the GPU
 * and hands out those Connectivity values for any block of cells, so a binding never builds the
 * P^2*K Job structs of resources.go:284-364. */
typedef enum { /* probe.Connectivity, in the order of AllConnectivity (connectivity.go:16-23) */
  CYC_CONN_UNKNOWN = 0,
  CYC_CONN_CHECK_FAILED = 1,
  CYC_CONN_INVALID_NAMED_PORT = 2,
  CYC_CONN_INVALID_PORT_PROTOCOL = 3,
  CYC_CONN_BLOCKED = 4,
  CYC_CONN_ALLOWED = 5,
  CYC_CONN_NO_JOB = 255 /* no job in this slot: the Item has no JobResult for it */
} cyc_connectivity;

typedef struct cyc_table cyc_table;

/* Run the probe for target rows [row_lo, row_hi) into planes the table owns (synchronous; panics
 * are reported as by cyc_probe_run).  A table stays valid after its context is destroyed. */
int cyc_table_run(cyc_ctx* ctx, int64_t row_lo, int64_t row_hi, cyc_table** out);
/* A table over planes the caller produced with cyc_probe_run (device pointers, not owned; they
 * must outlive the table and the run must be complete before cyc_table_cells). */
int cyc_table_wrap(cyc_ctx* ctx, const uint64_t* d_ingress, const uint64_t* d_egress, const uint8_t* d_status,
                   int64_t row_lo, int64_t row_hi, cyc_table** out);
/* The same under a row partition (cyc_probe_run_rows).  A CYC_ROWS_SOURCE table answers every cell
 * (s, d, k) with s inside its rows: Ingress, Egress and Combined of Table.Get(from = s, to = d). */
int cyc_table_run_rows(cyc_ctx* ctx, int partition, int64_t row_lo, int64_t row_hi, cyc_table** out);
int cyc_table_wrap_rows(cyc_ctx* ctx, const uint64_t* d_ingress, const uint64_t* d_egress, const uint8_t* d_status,
                        int partition, int64_t row_lo, int64_t row_hi, cyc_table** out);
/* Connectivity of every cell (s, d, k) of sources [s_lo,s_hi) x destinations [d_lo,d_hi) x slots
 * [k_lo,k_hi), computed on the device, into host arrays indexed
 *   ((s - s_lo) * (d_hi - d_lo) + (d - d_lo)) * (k_hi - k_lo) + (k - k_lo)
 * ingress / egress / combined are each optional (NULL = not wanted): JobResult.Ingress, .Egress and
 * .Combined of that job (jobrunner.go:36-55,85-93).  Target rows: ingress needs the destinations
 * inside the table's rows, egress the sources, combined both.  Source rows: every output needs the
 * sources inside the table's rows (any destination). */
int cyc_table_cells(cyc_table* t, int64_t s_lo, int64_t s_hi, int64_t d_lo, int64_t d_hi, int64_t k_lo, int64_t k_hi,
                    uint8_t* ingress, uint8_t* egress, uint8_t* combined);
/* out[0..7] = pods, slots, words, row_lo, row_hi, partition, ingress window first word, window words */
int cyc_table_shape(const cyc_table* t, int64_t* out, int n);
const char* cyc_table_error(const cyc_table* t);
void cyc_table_destroy(cyc_table* t);

/* ---- Multi-GPU table assembly over RCCL (north_star: "Source-pod rows shard across the 8 GPUs of one
 * node, with an RCCL all-gather over xGMI only to assemble the final table").  One process per GPU,
 * each with its own context.  The shards need no exchange (cyc_probe_run_rows); a Go multi-GPU
 * Runner.RunProbeForConfig (pkg/connectivity/probe/jobrunner.go:29-31) that returns a whole *Table on
 * every rank assembles it with these.  Rank 0 makes the unique id, the host hands its 128 bytes to
 * every rank by its own means (e.g. over the same channel that started the ranks), and every rank
 * calls cyc_comm_init with it; the context owns the communicator until cyc_comm_destroy or
 * cyc_ctx_destroy.  RCCL failures return CYC_ERR_RCCL with RCCL's message. */
#define CYC_COMM_ID_BYTES 128 /* ncclUniqueId */
int cyc_comm_unique_id(uint8_t* id);  /* id: CYC_COMM_ID_BYTES bytes (needs no context) */
int cyc_comm_init(cyc_ctx* ctx, int nranks, int rank, const uint8_t* id);  /* collective over the ranks */
int cyc_comm_destroy(cyc_ctx* ctx);
/* The library's partition of the prepared pods over nranks: rank `rank`'s rows [*row_lo, *row_hi)
 * under `partition` (target rows balanced to a row; source rows to a 64-pod word).  The all-gathers
 * below assume every rank ran exactly these rows. */
int cyc_rows_shard(cyc_ctx* ctx, int partition, int nranks, int rank, int64_t* row_lo, int64_t* row_hi);
/* Collective: every rank passes its shard planes (cyc_probe_run_rows output for its cyc_rows_shard
 * rows, complete on `hip_stream` or before) and receives the whole [P][K][W] ingress and egress
 * planes (cyc_probe_run's layout over rows [0, P)) in d_ingress_full / d_egress_full, enqueued on
 * `hip_stream` (asynchronous).  Row shares move by grouped RCCL broadcasts straight into place (in
 * place when a shard already sits at its rows of the full plane); a source partition's ingress slices
 * are gathered in ~256 MB chunks and scattered into whole rows by a HIP kernel (two scratch buffers
 * the context keeps).  The status plane is whole on every rank already (cyc_probe_run_rows). */
int cyc_planes_allgather(cyc_ctx* ctx, void* hip_stream, int partition, const uint64_t* d_ingress,
                         const uint64_t* d_egress, uint64_t* d_ingress_full, uint64_t* d_egress_full);
/* Collective, on a device-resident table: `shard` is this rank's cyc_table_run_rows /
 * cyc_table_wrap_rows table for its cyc_rows_shard rows; *out becomes a whole table (target rows
 * [0, P), planes it owns) answering Table.Get(from, to) for every pair on every rank.  Synchronous. */
int cyc_table_allgather(cyc_ctx* ctx, const cyc_table* shard, cyc_table** out);
/* One GPU, no communicator: the whole ingress plane from all nranks source shards' ingress slices
 * (d_slices[r] = rank r's [P][K][Wr_r] plane for its cyc_rows_shard source rows) — the relayout step of
 * cyc_planes_allgather on its own (enqueued on hip_stream). */
int cyc_rows_merge_sources(cyc_ctx* ctx, void* hip_stream, int nranks, const uint64_t* const* d_slices,
                           uint64_t* d_ingress_full);

/* ---- Batched independent problems ("blocks", SURVEY §8f row 3: the generate sweep's many small
 * probe problems, interpreter.go:137-148, in one pass).  Resources.Pods is cut into consecutive pod
 * ranges: block b = pods [block_end[b-1], block_end[b]) answering probe config block_config[b] (an
 * index into probes_json) over its OWN pods only — its table is the one Runner.RunProbeForConfig
 * would build for that problem alone.  The caller gives every block its own namespaces (a block's
 * policies live in them; cyclonus_amd/batch.py prefixes "<b>~"), which the library checks: a
 * namespace with pods in two blocks is refused.  Only intra-block cells are computed and written:
 * each class row covers its block's 64-pod words only, and block b's output is a slab of
 *   ingress[d][k][j], egress[s][k][j]   (pods of the block, slots of its config, j < ceil(n_b/64)),
 *   status[d][k]
 * with bit i of word j = the block's pod 64*j + i; slab offsets from cyc_blocks_layout. */
int cyc_probe_prepare_blocks(cyc_ctx* ctx, const char* probes_json, size_t len, const int64_t* block_end,
                             const int32_t* block_config, int64_t n_blocks, cyc_probe_shape* shape);
/* out[2*b], out[2*b+1] = block b's plane slab offset (64-bit words) and status offset (bytes);
 * out[2*n_blocks], out[2*n_blocks+1] = the totals (n >= 2 * (n_blocks + 1)). */
int cyc_blocks_layout(cyc_ctx* ctx, int64_t* out, int64_t n);
/* Run every block (device slabs, synchronous only when an input can panic).  block_status[b] (host,
 * optional) = the cyc_status block b's stand-alone run would end with: CYC_OK, or the reference's
 * panic / table-build fatal for THAT problem (its first panicking job in its own job order), with
 * the message in cyc_block_error(ctx, b).  Other blocks are unaffected by one block's panic. */
int cyc_probe_run_blocks(cyc_ctx* ctx, void* hip_stream, uint64_t* d_ingress, uint64_t* d_egress, uint8_t* d_status,
                         int32_t* block_status);
const char* cyc_block_error(const cyc_ctx* ctx, int64_t block);

/* Average device time (ms) of the last run's kernels, measured with HIP events on the launch
 * stream: [0] whole pipeline, [1] the emit launch (the HBM-roofline kernel; one launch writes both
 * planes), [2] class rows of both directions.  Eager runs ("graphs" = 0) always record them; graph
 * and fused-eager runs only with "step_events" = 1, and report only [0] ([1], [2] = -1); without
 * events the call fails with CYC_ERR_ARG. */
int cyc_last_timings(cyc_ctx* ctx, double* ms, int n);

/* Diagnostic: number of distinct classes (class rows computed) of the last run, [0] ingress,
 * [1] egress (synchronises the stream the last run was enqueued on, which must still exist). */
int cyc_last_classes(cyc_ctx* ctx, int64_t* out, int n);

/* What the last enqueued run's emit launched: the kernel name(s) ("k_emit_wide_buf<512,13>",
 * "k_emit_units<1024,7>", ...; several joined by " + ") into name (NUL-terminated, truncated to
 * cap - 1 bytes) and the number of emit launches into *launches (either may be null).  Set when the
 * run is enqueued (a captured graph replays what its capture recorded); CYC_ERR_ARG before any run. */
int cyc_last_emit(cyc_ctx* ctx, char* name, size_t cap, int64_t* launches);

/* Diagnostic path selectors (results never change; the GPU tests force every path):
 *   "graphs"      -1 (default: auto = 2 when the fused front applies, else 1); 1 replays the step as
 *                 one captured hipGraph when the inputs cannot panic (then cyc_last_timings reports
 *                 only the whole-pipeline time); 2 enqueues the same launches eagerly (the fused
 *                 front on the caller's stream, or the three-stream DAG); 0 runs every kernel in
 *                 order on the caller's stream with per-phase events
 *   "front_fused" 1 (default): the front as block-range-fused launches on one stream, one per
 *                 dependency level (no-panic builds with dense selectors); 0: the two-branch DAG
 *   "pod_words"   -1 (default: auto) / 0 / 1: class rows read pod-peer words from materialised peer
 *                 rows (0) or expand them from per-identity outcomes through each word's identity
 *                 runs (1, needs <= 4 runs per word and no possible panic)
 *   "pod_rows"    -1 (default: auto = 1 when identities >= pods / 2) / 0 / 1: materialised pod-peer
 *                 rows through identity outcomes and word runs (0) or per pod (1)
 *   "member_wave" -1 (default: auto = 1 for <= 4096 identities) / 0 / 1: target membership with a
 *                 thread (0) or a wave (1) per pod identity
 *   "class_rpb"   4 (default, 1..64): class representatives per identity-set class-row block
 *   "step_events" 0 (default) / 1: graph and fused-eager runs also record the whole-step timing
 *                 events cyc_last_timings reads (they idle the GPU ~9 us between steps)
 *   "pl_wave"     1 (default) / 0: materialised-row class rows a wave per 64-word chunk where they
 *                 fit (<= 4 job slots and descriptors), or a thread per (slot chunk, word) item
 *   "pr_group"    -1 (default: auto) / 1..64: the fused front's sparse pod-peer rows (PM builds) with
 *                 a block per pod peer (1) or a wave per 64-word chunk over groups of that many peers
 *   "class_inplace" -1 (default: auto) / 0 / 1: on the fused front, each class's rows are written
 *                 straight into the output planes at its first member pod's row and the emit copies
 *                 them to the class's other pods (1), or they go to a buffer of their own the emit
 *                 copies from (0); auto = 1 when the rows' identities are >= 1/16 of the rows or
 *                 the run is an identity-set build
 *   "sel_lazy"    -1 (default: auto) / 0 / 1: on the fused front, label selectors are evaluated where
 *                 membership and pod-peer rows / identity sets use them (1) instead of as the dense
 *                 selector x label-set table first (0); auto = 1 for identity-set builds and once
 *                 that table has >= 64M pairs
 *   "ip_iv"       -1 (default: auto) / 0: IP rows as pod-index intervals where the network's family holds
 *                 non-decreasing addresses in pod order (ip_rows_iv_blk), or through the paths below
 *   "ip_items"    -1 (default: auto = 1 for runs over every row) / 0 / 1: the fused front's IP rows as
 *                 per-chunk work items of the rows that touch each chunk (1) or as groups of 16 rows a
 *                 wave over 4 chunks (0)
 *   "emit_interleave" -1 (default: auto = 1 when a plane of a target-row run is >= 8 GB) / 0 / 1: the
 *                 emit's row list alternates ingress and egress rows (1) or holds all ingress rows first
 *   "row_phases"  -1 (default: auto = 2 for whole no-panic tables whose planes are >= 8 GB) / 1 / 2: the
 *                 class rows and the emit in two row phases (the classes rows [0, P/2) use, those rows'
 *                 emit, then the other classes and rows [P/2, P)) or in one pass (1); the fused front
 *                 runs once either way (phase 1's emit on a second stream under phase 2's class rows
 *                 was 4-7 % slower: profiles/r06_row_phases_ab.txt)
 * cyc_get_option also reports "launch" (the graphs mode in effect), "row_phases_active" (the last
 * run's phases: 2, or 0), "front_fused_active" and
 * "pl_wave_active" (all need cyc_probe_prepare); "pod_words" reports the mode the prepared probe
 * uses (0 or 1). */
int cyc_set_option(cyc_ctx* ctx, const char* name, int64_t value);
int cyc_get_option(cyc_ctx* ctx, const char* name, int64_t* value);

/* Single-cell API (policy.go:131-174): traffic_json is a JSON array of matcher.Traffic objects;
 * out[i] = ingress | egress << 1 (allowed bits).  Needs only a loaded policy. */
int cyc_query_traffic(cyc_ctx* ctx, const char* traffic_json, size_t len, uint8_t* out, int64_t n);

/* matcher.Traffic values (pkg/matcher/traffic.go:11-18) as flat tables, the form a cgo
 * SimulatedJobRunner.RunJobs over explicit []*Job (jobrunner.go:68-94, Job.Traffic job.go:81-103)
 * passes without JSON.  Endpoint 2i is traffic i's Source, 2i + 1 its Destination; an endpoint is
 * internal when internal[e] is 1 (TrafficPeer.Internal != nil: its namespace, pod labels and
 * namespace labels are read), external otherwise (only its IP).  A nil label map is given as an
 * empty range (the matchers read nil and empty maps alike); label_off / ns_label_off may be NULL
 * when no endpoint has labels. */
typedef struct {
  cyc_strings str;
  int64_t n;                         /* traffics */
  const uint8_t* internal;           /* [2n] */
  const int32_t* ip;                 /* [2n] TrafficPeer.IP */
  const int32_t* ns;                 /* [2n] Internal.Namespace (internal endpoints) */
  const int64_t* label_off;          /* [2n + 1] into label_key / label_val: Internal.PodLabels */
  const int32_t *label_key, *label_val;
  const int64_t* ns_label_off;       /* [2n + 1] into ns_label_key / ns_label_val: Internal.NamespaceLabels */
  const int32_t *ns_label_key, *ns_label_val;
  const int32_t* port;               /* [n] ResolvedPort */
  const int32_t* port_name;          /* [n] ResolvedPortName */
  const int32_t* protocol;           /* [n] Protocol (the raw string) */
} cyc_traffic_tables;
/* cyc_query_traffic over flat tables: out[i] = ingress | egress << 1; panics as cyc_query_traffic. */
int cyc_query_traffic_tables(cyc_ctx* ctx, const cyc_traffic_tables* tables, uint8_t* out, int64_t n);

/* query-traffic with the DirectionResult target lists (replaces Policy.IsTrafficAllowed's
 * AllowedResult, policy.go:84-96,131-174, as printed by analyze.go:209-225).  out_json gets a
 * JSON array, one object per traffic:
 *   {"Ingress": {"AllowingTargets": [pk, ...], "DenyingTargets": [pk, ...], "IsAllowed": b},
 *    "Egress": {...}, "IsAllowed": b}
 * pk = the target's primary key (target.go:57-62, the key of Policy.Ingress / Policy.Egress).
 * Lists are in primary-key order (Go walks the target map in random order).  *needed = bytes
 * required incl. the NUL; CYC_ERR_ARG when cap is smaller.  Panics as cyc_query_traffic. */
int cyc_query_traffic_targets(cyc_ctx* ctx, const char* traffic_json, size_t len, char* out_json, size_t cap,
                              size_t* needed);

/* query-target (analyze.go:163-204 QueryTargets / QueryTargetHelper): pods_json is a JSON list
 * of {"Namespace": ns, "Labels": {...}} (QueryTargetPod); out_json gets, per pod,
 * {"Ingress": [pk, ...], "Egress": [pk, ...]} = Policy.TargetsApplyingToPod (policy.go:68-82) per
 * direction, in primary-key order.  An invalid selector operator panics ("invalid operator"). */
int cyc_query_targets(cyc_ctx* ctx, const char* pods_json, size_t len, char* out_json, size_t cap, size_t* needed);

#ifdef __cplusplus
}
#endif
#endif /* CYCLONUS_HIP_H */
