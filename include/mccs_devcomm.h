/*
 * mccs_devcomm.h — device ABI shared between the mCCS host service and the
 * MI355X (gfx950) collective kernels.
 *
 * Layout-identical replacement for the reference's
 *   src/collectives/include/devcomm.h:36-163   (structs)
 *   src/collectives/include/devcomm.h:9-34     (constants)
 *   src/collectives/include/collectives.h:177-202 (dtype / redop enums)
 * which the Rust service imports through bindgen in
 *   src/collectives-sys/build.rs:21-36 (types ^mccsDev.*, vars ^MCCS.*).
 *
 * Written from scratch as plain C (also valid C++/HIP).  Every offset and size
 * is pinned by the static asserts at the bottom; the same numbers were dumped
 * from the reference header by oracle/ref_layout.cpp and are checked again by
 * tests/test_abi_layout.py against tests/golden/abi_layout.json.
 *
 * WARP_SIZE stays 32 because it is part of the ABI: the host expresses block
 * sizes as nWarps 32-lane units (plan.rs:41,182).  The gfx950 kernels run
 * 64-lane wavefronts internally and only use nWarps*32 for the reference's
 * chunk-size arithmetic (all_reduce.h:30-36).
 */
#ifndef MCCS_AMD_DEVCOMM_H_
#define MCCS_AMD_DEVCOMM_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- constants (devcomm.h:9-34, collectives.h:270-274) ------------------ */
#define MCCS_NUM_FUNCTIONS 5
#define MCCS_NUM_ALGORITHMS 1
#define MCCS_ALGO_RING 0
#define MCCS_NUM_PROTOCOLS 1
#define MCCS_PROTO_SIMPLE 0
#define MCCS_MAX_OPS 2048
#define MCCS_BUFFER_SLOTS 8
#define WARP_SIZE 32
#define MCCS_MAX_NCHANNELS 32
#define MCCS_MAX_NTHREADS 640
#define MCCS_SIMPLE_MAX_NTHREADS 512
#define MCCS_MAX_CONNS 2
#define MCCS_WORK_SIZE 512
#define MCCS_MAX_WORK_ELEMENTS 10
#define MCCS_MAX_WORK_ELEMENTS_P2P 16
#define MCCS_MAX_GROUPS 16

#define ALLGATHER_SLICESTEPS (MCCS_BUFFER_SLOTS / 4)
#define ALLGATHER_CHUNKSTEPS (MCCS_BUFFER_SLOTS / 2)
#define ALLREDUCE_SLICESTEPS (MCCS_BUFFER_SLOTS / 4)
#define ALLREDUCE_CHUNKSTEPS (MCCS_BUFFER_SLOTS / 2)
#define MCCS_MAX_SLICE_PER_CHUNK 2

/* ---- enums ---------------------------------------------------------------- */
typedef enum {
  mccsFuncBoadcast = 0, /* sic, reference spelling (devcomm.h:11) */
  mccsFuncReduce = 1,
  mccsFuncAllGather = 2,
  mccsFuncReduceScatter = 3,
  mccsFuncAllReduce = 4,
  mccsFuncSendRecv = 5,
  mccsFuncSend = 6,
  mccsFuncRecv = 7,
  mccsNumFuncs = 8
} mccsDevFunc_t;

/* collectives.h:177-192 (bf16 present: the CUDA >= 11 layout) */
typedef enum {
  mccsInt8 = 0,
  mccsChar = 0,
  mccsUint8 = 1,
  mccsInt32 = 2,
  mccsInt = 2,
  mccsUint32 = 3,
  mccsInt64 = 4,
  mccsUint64 = 5,
  mccsFloat16 = 6,
  mccsHalf = 6,
  mccsFloat32 = 7,
  mccsFloat = 7,
  mccsFloat64 = 8,
  mccsDouble = 8,
  mccsBfloat16 = 9,
  mccsNumTypes = 10
} mccsDevDataType_t;

/* collectives.h:194-198 */
typedef enum {
  mccsDevSum = 0,
  mccsDevProd = 1,
  mccsDevMax = 2,
  mccsDevMin = 3,
  mccsDevPreMulSum = 4,
  mccsDevSumPostDiv = 5,
  mccsNumDevRedOps = 6
} mccsDevRedOp_t;

/* devcomm.h:67-76: C++ enums with uint8_t storage; plain uint8_t here so the
 * header stays valid C.  Values are identical. */
typedef uint8_t mccsDevWorkType_t;
#define mccsDevWorkTypeUnused ((mccsDevWorkType_t)0)
#define mccsDevWorkTypeColl ((mccsDevWorkType_t)1)
#define mccsDevWorkTypeP2p ((mccsDevWorkType_t)2)

/* ---- structs (devcomm.h:36-163) ----------------------------------------- */

/* One direction of a FIFO connection.  Receiver polls *tail and posts *head;
 * sender polls *head and posts *tail (prims_simple.h:68-125). */
struct mccsDevConnInfo {
  char *buffs[MCCS_NUM_PROTOCOLS]; /* FIFO data: MCCS_BUFFER_SLOTS steps */
  uint64_t *tail;                  /* local for recv, remote for send */
  uint64_t *head;                  /* local for send, remote for recv */
  int *sizesFifo;                  /* optional per-slot byte counts */
  int *offsFifo;                   /* unused (NULL) in mCCS */
  uint64_t step;                   /* persists across launches */
};

struct mccsDevRing {
  int prev;
  int next;
  int *userRanks; /* ring order starting at this rank */
  int index;      /* this rank's distance from rank 0 along the ring */
};

struct mccsDevWorkHeader {
  union {
    int32_t workNext;  /* isLast == 0: offset (in works) from workHead */
    uint32_t doneAcks; /* isLast == 1: value written to *workFifoDone */
  };
  uint16_t funcIndex;
  uint8_t isLast : 1;
  uint8_t inFifo : 1;
  mccsDevWorkType_t type;
};

struct mccsDevWorkElem {
  uint8_t isUsed : 1;
  uint8_t nWarps; /* block size in 32-lane units as the host computed it */
  const void *sendbuff;
  void *recvbuff;
  size_t count; /* elements of the collective's dtype */
  uint32_t root;
  uint8_t bid;       /* index of this channel among the plan's channels */
  uint8_t nChannels; /* channels sharing this collective */
  uint64_t redOpArg;
};

struct mccsDevWorkElemP2p {
  int peer : 30;
  int proto : 2;
  uint8_t p2pType;
  uint8_t nWarps;
  uint8_t warpStart;
  uint8_t ngroups;
  uint32_t buffHi32, buffLo32;
  uint32_t countHi32, countLo32;
  int chunkSize;
};

struct mccsDevWork {
  struct mccsDevWorkHeader header;
  union {
    char pad[MCCS_WORK_SIZE - sizeof(struct mccsDevWorkHeader)];
    struct mccsDevWorkElem elems[MCCS_MAX_WORK_ELEMENTS];
    struct mccsDevWorkElemP2p p2pElems[MCCS_MAX_WORK_ELEMENTS_P2P];
  };
};

struct mccsDevChannelPeer {
  struct mccsDevConnInfo send[MCCS_MAX_CONNS];
  struct mccsDevConnInfo recv[MCCS_MAX_CONNS];
};

struct mccsDevChannel {
  struct mccsDevChannelPeer *peers; /* indexed by peer rank */
  struct mccsDevRing ring;
  uint32_t *workFifoDone;
} __attribute__((aligned(16)));

struct mccsDevComm {
  int rank;
  int nRanks;
  int buffSizes[MCCS_NUM_PROTOCOLS];
  volatile uint32_t *abortFlag;
};

struct mccsDevCommAndChannels {
  struct mccsDevComm comm;
  struct mccsDevChannel channels[MCCS_MAX_NCHANNELS];
} __attribute__((aligned(16)));

/* ---- pinned layout (golden values from oracle/ref_layout.cpp) ----------- */
#ifdef __cplusplus
#define MCCS_STATIC_ASSERT(c, m) static_assert(c, m)
#else
#define MCCS_STATIC_ASSERT(c, m) _Static_assert(c, m)
#endif

MCCS_STATIC_ASSERT(sizeof(struct mccsDevConnInfo) == 48, "ConnInfo size");
MCCS_STATIC_ASSERT(offsetof(struct mccsDevConnInfo, tail) == 8, "ConnInfo.tail");
MCCS_STATIC_ASSERT(offsetof(struct mccsDevConnInfo, head) == 16, "ConnInfo.head");
MCCS_STATIC_ASSERT(offsetof(struct mccsDevConnInfo, sizesFifo) == 24, "ConnInfo.sizesFifo");
MCCS_STATIC_ASSERT(offsetof(struct mccsDevConnInfo, offsFifo) == 32, "ConnInfo.offsFifo");
MCCS_STATIC_ASSERT(offsetof(struct mccsDevConnInfo, step) == 40, "ConnInfo.step");
MCCS_STATIC_ASSERT(sizeof(struct mccsDevRing) == 24, "Ring size");
MCCS_STATIC_ASSERT(offsetof(struct mccsDevRing, userRanks) == 8, "Ring.userRanks");
MCCS_STATIC_ASSERT(offsetof(struct mccsDevRing, index) == 16, "Ring.index");
MCCS_STATIC_ASSERT(sizeof(struct mccsDevWorkHeader) == 8, "WorkHeader size");
MCCS_STATIC_ASSERT(offsetof(struct mccsDevWorkHeader, funcIndex) == 4, "WorkHeader.funcIndex");
MCCS_STATIC_ASSERT(offsetof(struct mccsDevWorkHeader, type) == 7, "WorkHeader.type");
MCCS_STATIC_ASSERT(sizeof(struct mccsDevWorkElem) == 48, "WorkElem size");
MCCS_STATIC_ASSERT(offsetof(struct mccsDevWorkElem, nWarps) == 1, "WorkElem.nWarps");
MCCS_STATIC_ASSERT(offsetof(struct mccsDevWorkElem, sendbuff) == 8, "WorkElem.sendbuff");
MCCS_STATIC_ASSERT(offsetof(struct mccsDevWorkElem, recvbuff) == 16, "WorkElem.recvbuff");
MCCS_STATIC_ASSERT(offsetof(struct mccsDevWorkElem, count) == 24, "WorkElem.count");
MCCS_STATIC_ASSERT(offsetof(struct mccsDevWorkElem, root) == 32, "WorkElem.root");
MCCS_STATIC_ASSERT(offsetof(struct mccsDevWorkElem, bid) == 36, "WorkElem.bid");
MCCS_STATIC_ASSERT(offsetof(struct mccsDevWorkElem, nChannels) == 37, "WorkElem.nChannels");
MCCS_STATIC_ASSERT(offsetof(struct mccsDevWorkElem, redOpArg) == 40, "WorkElem.redOpArg");
MCCS_STATIC_ASSERT(sizeof(struct mccsDevWorkElemP2p) == 28, "WorkElemP2p size");
MCCS_STATIC_ASSERT(sizeof(struct mccsDevWork) == MCCS_WORK_SIZE, "Work size");
MCCS_STATIC_ASSERT(offsetof(struct mccsDevWork, elems) == 8, "Work.elems");
MCCS_STATIC_ASSERT(sizeof(struct mccsDevChannelPeer) == 192, "ChannelPeer size");
MCCS_STATIC_ASSERT(offsetof(struct mccsDevChannelPeer, recv) == 96, "ChannelPeer.recv");
MCCS_STATIC_ASSERT(sizeof(struct mccsDevChannel) == 48, "Channel size");
MCCS_STATIC_ASSERT(offsetof(struct mccsDevChannel, ring) == 8, "Channel.ring");
MCCS_STATIC_ASSERT(offsetof(struct mccsDevChannel, workFifoDone) == 32, "Channel.workFifoDone");
MCCS_STATIC_ASSERT(sizeof(struct mccsDevComm) == 24, "Comm size");
MCCS_STATIC_ASSERT(offsetof(struct mccsDevComm, buffSizes) == 8, "Comm.buffSizes");
MCCS_STATIC_ASSERT(offsetof(struct mccsDevComm, abortFlag) == 16, "Comm.abortFlag");
MCCS_STATIC_ASSERT(sizeof(struct mccsDevCommAndChannels) == 1568, "CommAndChannels size");
MCCS_STATIC_ASSERT(offsetof(struct mccsDevCommAndChannels, channels) == 32, "CommAndChannels.channels");

#ifdef __cplusplus
}
#endif

#endif /* MCCS_AMD_DEVCOMM_H_ */
