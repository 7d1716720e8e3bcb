// tables.h — POD layouts of the flattened policy / probe tables shared by the host compiler
// (host.cpp) and the CDNA4 kernels (engine.hip).  All fields are 32-bit so every record is a
// multiple of 16 bytes and loads as dwordx4.
#pragma once
#include <stdint.h>

// Label-selector requirement (pkg/kube/labelselector.go:24-86).
enum {
  REQ_EQ = 0,        // matchLabels k:v, v != ""      -> labels[k] == v
  REQ_EQ_EMPTY = 1,  // matchLabels k:"" -> labels[k] == "" (TRUE when k is absent, :70)
  REQ_IN = 2,        // key present && value in set
  REQ_NOTIN = 3,     // key present && value not in set (absent key => false, :37-42)
  REQ_EXISTS = 4,
  REQ_DNE = 5,
  REQ_INVALID = 6,  // unknown operator: panic("invalid operator") when reached (:57)
};
typedef struct {
  uint32_t op, key, voff, vcnt;  // values = req_vals[voff .. voff+vcnt)
} DReq;

// net.IP after Go's To4 collapse: fam 4 uses w[3] only; fam 6 uses w[0..3]. valid=0: unparsable.
typedef struct {
  uint32_t valid, fam, pad0, pad1;
  uint32_t w[4];
} DIP;

// *net.IPNet after networkNumberAndMask: fam 4 => net/mask in [3]; fam 6 => all four words.
typedef struct {
  uint32_t valid, fam, pad0, pad1;
  uint32_t net[4], mask[4];
} DCidr;

typedef struct {
  uint32_t cidr, exoff, excnt, pad;  // excepts = ipb_ex[exoff .. exoff+excnt) (cidr ids)
} DIPBlock;

// Port matcher entries (pkg/matcher/portmatcher.go).
enum { PE_PROTO = 0, PE_INT = 1, PE_NAME = 2, PE_RANGE = 3 };
typedef struct {
  uint32_t kind;
  int32_t a, b;    // PE_INT: a = port; PE_NAME: a = name id; PE_RANGE: [a, b]
  uint32_t proto;  // protocol string id (raw string compare)
} DPortEntry;
typedef struct {
  uint32_t all, eoff, ecnt, pad;
} DPortM;

// Peer matcher.  kind: 0 AllPeers, 1 PortsForAllPeers, 2 PodPeer, 3 IPPeer.
// nskind: 0 exact (nsval = namespace string id), 1 all, 2 label selector (nsval = selector id).
typedef struct {
  uint32_t kind, port, nskind, nsval, podsel, ipb, pad0, pad1;  // podsel == CYC_ALL => all pods
} DPeer;
#define CYC_ALL 0xFFFFFFFFu

typedef struct {
  uint32_t ns, sel, poff, pcnt;  // peers = peers[poff .. poff+pcnt), slice order
} DTarget;

// Job descriptor (Traffic.ResolvedPort / ResolvedPortName / Protocol).
typedef struct {
  int32_t port;
  uint32_t name, proto, pad;
} DDesc;
