/*
 * kubeapi_oracle.c — CPU ORACLE (TEST INFRASTRUCTURE ONLY; see header).
 *
 * A deliberately plain, sequential restatement of KubeAPI.tla's TLA+
 * translation (/root/reference/KubeAPI.tla:373-789) explored by a FIFO
 * breadth-first search with TLC's successor-enumeration semantics
 * (SURVEY.md Appendix A):
 *   - Next is split into 22 actions; each is evaluated for every `self` of
 *     its quantifier domain, in the order of the Next disjunction
 *     (KubeAPI.tla:760-763);
 *   - every disjunct is a branch, including constant-only disjuncts
 *     (REQUESTS_CAN_FAIL \/ REQUESTS_CAN_TIMEOUT, :476,504) and
 *     `TRUE /\ UNCHANGED` (:487,515) — duplicates are all "generated";
 *   - IF/THEN/ELSE does not branch; \E x \in S branches once per element;
 *   - Assert(FALSE, ...) inside an action is an evaluation error raised while
 *     the state is being expanded (TLC reports the trace up to that state);
 *   - invariants are checked on every new distinct state (MC.cfg:13-15);
 *   - deadlock = a state with no successor (launch:16).
 *
 * State representation: the "canonical tuple" of DESIGN.md §3 — one byte
 * (or one mask) per TLA+ sub-value, every unused field zero, so equal TLA+
 * values <=> equal bytes.  Dedup uses 128-bit fingerprints of those bytes
 * (two independent 64-bit hashes), i.e. exact for all practical purposes.
 * This representation is intentionally NOT the product's packed layout.
 */
#include "kubeapi_oracle.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ---------------------------------------------------------------- values */
/* TLA+ strings used as op values (KubeAPI.tla:415 Verbs) */
enum { OP_DIV = 0, OP_Create, OP_Get, OP_Update, OP_Delete, OP_Force };
/* Responses (KubeAPI.tla:421) */
enum { ST_NONE = 0, ST_Pending, ST_Ok, ST_Error };
/* kind values: defaultInitValue, "Secret", "PVC" */
enum { K_DIV = 0, K_Secret, K_PVC };
/* stack frame procedure */
enum { PR_NONE = 0, PR_API, PR_ListAPI };
/* object identities: [k |-> "Secret", n |-> "foo"], [k |-> "PVC", n |-> "mypvc"]
 * (KubeAPI.tla:176,182,188) */
enum { ID_SECRET = 0, ID_PVC = 1 };

/* An object value ("oval"): one byte.
 *   bit0 def    : 1 = a record, 0 = defaultInitValue (MC.cfg:2)
 *   bit1 id     : identity (k,n)
 *   bit2 has_vv : "vv" \in DOMAIN o
 *   bit3 spec   : "spec" \in DOMAIN o (always [pvname |-> o.n] when present)
 *   bit4-7 vv   : the version vector, a set of reader processes          */
typedef uint8_t oval;
#define OV_DEF 1u
#define OV_ID(o) (((o) >> 1) & 1u)
#define OV_HASVV(o) (((o) >> 2) & 1u)
#define OV_SPEC(o) (((o) >> 3) & 1u)
#define OV_VV(o) (((o) >> 4) & 0xFu)
/* lostUpdate, the history variable of the build-defined NoLostUpdate, kept
 * in bit 63 of kstate.api (see check_invariants) */
#define KO_LOST_UPDATE (1ull << 63)
static inline oval ov_bare(int id) { return (oval)(OV_DEF | (id << 1)); }
static inline oval ov_make(int id, int hasvv, int spec, int vv) {
  return (oval)(OV_DEF | (id << 1) | (hasvv << 2) | (spec << 3) | (vv << 4));
}

typedef struct {
  uint64_t api;                /* apiState as a set over U (bitmask) */
  uint64_t lr_objs[KO_MAXP];   /* listRequests[p].objs, set over U */
  uint8_t pc[KO_MAXP];
  uint8_t op[KO_MAXP];
  oval obj[KO_MAXP];
  uint8_t kind[KO_MAXP];
  uint8_t sr[KO_MAXP];         /* shouldReconcile[p] (clients only) */
  uint8_t sdepth[KO_MAXP];     /* Len(stack[p]) */
  uint8_t sproc[KO_MAXP];      /* Head(stack[p]).procedure */
  uint8_t spc[KO_MAXP];        /* Head(stack[p]).pc */
  uint8_t sop[KO_MAXP];        /* Head(stack[p]).op   (API frames) */
  oval sobj[KO_MAXP];          /* Head(stack[p]).obj  (API frames) */
  uint8_t skind[KO_MAXP];      /* Head(stack[p]).kind (ListAPI frames) */
  uint8_t rq_present[KO_MAXP]; /* p \in DOMAIN requests */
  uint8_t rq_op[KO_MAXP];
  uint8_t rq_status[KO_MAXP];
  oval rq_obj[KO_MAXP];
  uint8_t lr_present[KO_MAXP]; /* p \in DOMAIN listRequests */
  uint8_t lr_kind[KO_MAXP];
  uint8_t lr_status[KO_MAXP];
  uint8_t pad[6];
} kstate;

/* ------------------------------------------------------------ model ctx */
typedef struct {
  ko_config cfg;
  int P, R;                   /* processes, readers (clients + controllers) */
  uint64_t idmask[2];         /* U bits of each identity */
  uint64_t allmask;
} model;

enum { PK_CLIENT, PK_PVC, PK_SERVER };
static int pkind(const model *m, int p) {
  if (p < m->cfg.nc) return PK_CLIENT;
  if (p < m->cfg.nc + m->cfg.np) return PK_PVC;
  return PK_SERVER;
}

/* U index of an apiState element: id<<(R+1) | spec<<R | vv */
static inline int u_of(const model *m, oval o) {
  return (OV_ID(o) << (m->R + 1)) | (OV_SPEC(o) << m->R) | OV_VV(o);
}
static inline oval ov_of_u(const model *m, int u) {
  int id = (u >> (m->R + 1)) & 1, spec = (u >> m->R) & 1, vv = u & ((1 << m->R) - 1);
  return ov_make(id, 1, spec, vv);
}

static void model_init(model *m, const ko_config *cfg) {
  memset(m, 0, sizeof *m);
  m->cfg = *cfg;
  m->P = cfg->nc + cfg->np + cfg->ns;
  m->R = cfg->nc + cfg->np;
  if (m->P > KO_MAXP || m->R > 4 || m->R < 1) {
    fprintf(stderr, "kubeapi_oracle: unsupported NC/NP/NS\n");
    abort();
  }
  int usz = 1 << (m->R + 1);
  for (int u = 0; u < 2 * usz; u++) m->idmask[u / usz] |= 1ull << u;
  m->allmask = m->idmask[0] | m->idmask[1];
}

/* ------------------------------------------------------------- helpers */
/* Write(o) == "vv" :> {} @@ o   (KubeAPI.tla:395) */
static inline oval tla_Write(oval o) { return (oval)((o & 0x0F) | (1u << 2)); }
/* Read(o, c) == [o EXCEPT !.vv = @ \cup {c}]   (KubeAPI.tla:399) */
static inline oval tla_Read(oval o, int c) { return (oval)(o | (1u << (4 + c))); }
/* HasRead(o, c) == c \in o.vv   (KubeAPI.tla:404) */
static inline int tla_HasRead(oval o, int c) { return (OV_VV(o) >> c) & 1; }
/* ObjectExists(obj) == \E o \in apiState: IsVersionOf(o, obj)  (:410) */
static inline int tla_ObjectExists(const model *m, const kstate *s, int id) {
  return (s->api & m->idmask[id]) != 0;
}
/* IsUnboundPVC(pvc) (:444-446): k = "PVC" /\ ("spec" \notin DOMAIN pvc \/ ...) */
static inline int tla_IsUnboundPVC(oval o) { return OV_ID(o) == ID_PVC && !OV_SPEC(o); }
/* o.k of identity */
static inline int kind_of_id(int id) { return id == ID_SECRET ? K_Secret : K_PVC; }

static int popc64(uint64_t x) { return __builtin_popcountll(x); }

/* branch counters: KO_B_* in the header */
#define NBRANCH KO_NBRANCH

/* ---------------------------------------------------- successor emitter */
typedef struct {
  kstate *succ;      /* output array */
  uint8_t *act;      /* action id per successor */
  int n, cap;
  int fail_action;   /* assertion failure: action id, else -1 */
  int fail_self;
  uint64_t *branch;  /* NBRANCH counters, may be NULL */
} emitter;

static inline void emit(emitter *e, const kstate *t, int a) {
  if (e->n >= e->cap) { fprintf(stderr, "kubeapi_oracle: successor overflow\n"); abort(); }
  e->succ[e->n] = *t;
  e->act[e->n] = (uint8_t)a;
  e->n++;
}
static inline void br(emitter *e, int b) { if (e->branch) e->branch[b]++; }

/* push an API frame (KubeAPI.tla:535-539 and friends) */
static inline void push_api(kstate *t, int self, int retpc) {
  if (t->sdepth[self] != 0) { fprintf(stderr, "kubeapi_oracle: nested call\n"); abort(); }
  t->sdepth[self] = 1; t->sproc[self] = PR_API; t->spc[self] = (uint8_t)retpc;
  t->sop[self] = t->op[self]; t->sobj[self] = t->obj[self]; t->skind[self] = 0;
}
static inline void push_list(kstate *t, int self, int retpc) {
  if (t->sdepth[self] != 0) { fprintf(stderr, "kubeapi_oracle: nested call\n"); abort(); }
  t->sdepth[self] = 1; t->sproc[self] = PR_ListAPI; t->spc[self] = (uint8_t)retpc;
  t->sop[self] = 0; t->sobj[self] = 0; t->skind[self] = t->kind[self];
}
static inline void pop_frame(kstate *t, int self) {
  t->sdepth[self] = 0; t->sproc[self] = 0; t->spc[self] = 0;
  t->sop[self] = 0; t->sobj[self] = 0; t->skind[self] = 0;
}

/* ------------------------------------------------------- the 22 actions */
/* DoRequest(self)  KubeAPI.tla:471-483 */
static void a_DoRequest(const model *m, const kstate *s, int self, emitter *e) {
  if (s->pc[self] != KO_DoRequest) return;
  kstate t = *s;
  t.rq_present[self] = 1; t.rq_op[self] = s->op[self]; t.rq_obj[self] = s->obj[self];
  t.pc[self] = KO_DoReply;
  t.rq_status[self] = ST_Pending; emit(e, &t, 0);               /* :472-475 */
  t.rq_status[self] = ST_Error;                                  /* :476-480 */
  if (m->cfg.can_fail) emit(e, &t, 0);
  if (m->cfg.can_timeout) emit(e, &t, 0);
}
/* DoReply(self)  KubeAPI.tla:485-495 */
static void a_DoReply(const model *m, const kstate *s, int self, emitter *e) {
  if (s->pc[self] != KO_DoReply) return;
  if (!s->rq_present[self] || s->sdepth[self] != 1 || s->sproc[self] != PR_API) {
    fprintf(stderr, "kubeapi_oracle: DoReply eval error\n"); abort();
  }
  if (s->rq_status[self] == ST_Pending) return;                  /* :486 */
  kstate t = *s;
  t.pc[self] = s->spc[self]; t.op[self] = s->sop[self]; t.obj[self] = s->sobj[self];
  pop_frame(&t, self);
  emit(e, &t, 1);                                                /* :487-488 */
  if (m->cfg.can_timeout) { t.rq_status[self] = ST_Error; emit(e, &t, 1); } /* :489-490 */
}
/* DoListRequest(self)  KubeAPI.tla:499-511 */
static void a_DoListRequest(const model *m, const kstate *s, int self, emitter *e) {
  if (s->pc[self] != KO_DoListRequest) return;
  kstate t = *s;
  t.lr_present[self] = 1; t.lr_kind[self] = s->kind[self]; t.lr_objs[self] = 0;
  t.pc[self] = KO_DoListReply;
  t.lr_status[self] = ST_Pending; emit(e, &t, 2);
  t.lr_status[self] = ST_Error;
  if (m->cfg.can_fail) emit(e, &t, 2);
  if (m->cfg.can_timeout) emit(e, &t, 2);
}
/* DoListReply(self)  KubeAPI.tla:513-524 */
static void a_DoListReply(const model *m, const kstate *s, int self, emitter *e) {
  if (s->pc[self] != KO_DoListReply) return;
  if (!s->lr_present[self] || s->sdepth[self] != 1 || s->sproc[self] != PR_ListAPI) {
    fprintf(stderr, "kubeapi_oracle: DoListReply eval error\n"); abort();
  }
  if (s->lr_status[self] == ST_Pending) return;
  kstate t = *s;
  t.pc[self] = s->spc[self]; t.kind[self] = s->skind[self];
  pop_frame(&t, self);
  emit(e, &t, 3);
  if (m->cfg.can_timeout) { t.lr_objs[self] = 0; t.lr_status[self] = ST_Error; emit(e, &t, 3); }
}
/* CStart(self)  KubeAPI.tla:528-549 */
static void a_CStart(const model *m, const kstate *s, int self, emitter *e) {
  (void)m;
  if (s->pc[self] != KO_CStart) return;
  for (int b = 0; b < 2; b++) {
    kstate t = *s;
    if (b == 0) t.sr[self] = 1;                                  /* :529 */
    if (t.sr[self]) {                                            /* :532 primed read */
      br(e, KO_B_CSTART_THEN);
      push_api(&t, self, KO_C1);
      t.obj[self] = ov_bare(ID_SECRET); t.op[self] = OP_Force;
      t.pc[self] = KO_DoRequest;
    } else {
      br(e, KO_B_CSTART_ELSE);
      push_list(&t, self, KO_C3);
      t.kind[self] = K_Secret;
      t.pc[self] = KO_DoListRequest;
    }
    emit(e, &t, 4);
  }
}
static void a_C1(const model *m, const kstate *s, int self, emitter *e) {  /* :551-556 */
  if (s->pc[self] != KO_C1) return;
  kstate t = *s;
  /* variant 3 (seeded bug): the Force reply status is ignored, so C2's
   * Assert(ObjectExists(Secret)) (:598-599) can fail */
  if (s->rq_status[self] != ST_Ok && m->cfg.variant != 3) { br(e, KO_B_C1_START); t.pc[self] = KO_CStart; }
  else { br(e, KO_B_C1_C10); t.pc[self] = KO_C10; }
  emit(e, &t, 5);
}
static void a_C10(const model *m, const kstate *s, int self, emitter *e) { /* :558-568 */
  (void)m;
  if (s->pc[self] != KO_C10) return;
  kstate t = *s;
  push_api(&t, self, KO_C11);
  t.obj[self] = ov_bare(ID_PVC); t.op[self] = OP_Force; t.pc[self] = KO_DoRequest;
  emit(e, &t, 6);
}
static void a_C11(const model *m, const kstate *s, int self, emitter *e) { /* :570-575 */
  (void)m;
  if (s->pc[self] != KO_C11) return;
  kstate t = *s;
  if (s->rq_status[self] != ST_Ok) { br(e, KO_B_C11_START); t.pc[self] = KO_CStart; }
  else { br(e, KO_B_C11_c12); t.pc[self] = KO_c12; }
  emit(e, &t, 7);
}
static void a_c12(const model *m, const kstate *s, int self, emitter *e) { /* :577-587 */
  (void)m;
  if (s->pc[self] != KO_c12) return;
  kstate t = *s;
  push_api(&t, self, KO_C13);
  t.obj[self] = ov_bare(ID_PVC); t.op[self] = OP_Get; t.pc[self] = KO_DoRequest;
  emit(e, &t, 8);
}
static void a_C13(const model *m, const kstate *s, int self, emitter *e) { /* :589-594 */
  (void)m;
  if (s->pc[self] != KO_C13) return;
  kstate t = *s;
  int cond = s->rq_status[self] != ST_Ok;
  if (!cond) {
    if (!(s->rq_obj[self] & OV_DEF)) { fprintf(stderr, "kubeapi_oracle: C13 eval\n"); abort(); }
    cond = tla_IsUnboundPVC(s->rq_obj[self]);
  }
  if (cond) { br(e, KO_B_C13_START); t.pc[self] = KO_CStart; }
  else { br(e, KO_B_C13_C2); t.pc[self] = KO_C2; }
  emit(e, &t, 9);
}
static void a_C2(const model *m, const kstate *s, int self, emitter *e) { /* :596-602 */
  if (s->pc[self] != KO_C2) return;
  kstate t = *s;
  t.sr[self] = 0;                                                 /* :597 */
  if (!tla_ObjectExists(m, s, ID_SECRET)) {                       /* :598-599 */
    e->fail_action = 10; e->fail_self = self; return;
  }
  t.pc[self] = KO_C5;
  emit(e, &t, 10);
}
static void a_C3(const model *m, const kstate *s, int self, emitter *e) { /* :604-609 */
  (void)m;
  if (s->pc[self] != KO_C3) return;
  kstate t = *s;
  if (s->lr_status[self] != ST_Ok) { br(e, KO_B_C3_START); t.pc[self] = KO_CStart; }
  else { br(e, KO_B_C3_C8); t.pc[self] = KO_C8; }
  emit(e, &t, 11);
}
static void a_C8(const model *m, const kstate *s, int self, emitter *e) { /* :611-616 */
  (void)m;
  if (s->pc[self] != KO_C8) return;
  kstate t = *s;
  if (s->lr_objs[self] == 0) { br(e, KO_B_C8_C4); t.pc[self] = KO_C4; }
  else { br(e, KO_B_C8_C6); t.pc[self] = KO_C6; }
  emit(e, &t, 12);
}
static void a_C6(const model *m, const kstate *s, int self, emitter *e) { /* :618-629 */
  if (s->pc[self] != KO_C6) return;
  uint64_t objs = s->lr_objs[self];
  while (objs) {                                 /* \E s \in objs, U order */
    int u = __builtin_ctzll(objs); objs &= objs - 1;
    oval so = ov_of_u(m, u);
    kstate t = *s;
    push_api(&t, self, KO_C7);
    t.obj[self] = ov_bare(OV_ID(so));           /* [k |-> s.k, n |-> s.n] */
    t.op[self] = OP_Delete; t.pc[self] = KO_DoRequest;
    emit(e, &t, 13);
  }
}
static void a_C7(const model *m, const kstate *s, int self, emitter *e) { /* :631-636 */
  (void)m;
  if (s->pc[self] != KO_C7) return;
  kstate t = *s;
  if (s->rq_status[self] != ST_Ok || popc64(s->lr_objs[self]) > 1) {
    br(e, KO_B_C7_START); t.pc[self] = KO_CStart;
  } else { br(e, KO_B_C7_C4); t.pc[self] = KO_C4; }
  emit(e, &t, 14);
}
static void a_C4(const model *m, const kstate *s, int self, emitter *e) { /* :638-643 */
  if (s->pc[self] != KO_C4) return;
  if (tla_ObjectExists(m, s, ID_SECRET)) {                         /* :639-640 */
    e->fail_action = 15; e->fail_self = self; return;
  }
  kstate t = *s;
  t.pc[self] = KO_C5;
  emit(e, &t, 15);
}
static void a_C5(const model *m, const kstate *s, int self, emitter *e) { /* :645-648 */
  (void)m;
  if (s->pc[self] != KO_C5) return;
  kstate t = *s;
  t.pc[self] = KO_CStart;
  emit(e, &t, 16);
}
static void a_PVCStart(const model *m, const kstate *s, int self, emitter *e) { /* :655-663 */
  (void)m;
  if (s->pc[self] != KO_PVCStart) return;
  kstate t = *s;
  push_list(&t, self, KO_PVCListedPVCs);
  t.kind[self] = K_PVC; t.pc[self] = KO_DoListRequest;
  emit(e, &t, 17);
}
static uint64_t unbound_of(const model *m, uint64_t objs) {
  uint64_t r = 0;
  while (objs) {
    int u = __builtin_ctzll(objs); objs &= objs - 1;
    if (tla_IsUnboundPVC(ov_of_u(m, u))) r |= 1ull << u;
  }
  return r;
}
static void a_PVCListedPVCs(const model *m, const kstate *s, int self, emitter *e) { /* :665-671 */
  if (s->pc[self] != KO_PVCListedPVCs) return;
  kstate t = *s;
  if (s->lr_status[self] != ST_Ok || unbound_of(m, s->lr_objs[self]) == 0) {
    br(e, KO_B_PVCL_START); t.pc[self] = KO_PVCStart;
  } else { br(e, KO_B_PVCL_HAVE); t.pc[self] = KO_PVCHavePVCs; }
  emit(e, &t, 18);
}
static void a_PVCHavePVCs(const model *m, const kstate *s, int self, emitter *e) { /* :673-688 */
  if (s->pc[self] != KO_PVCHavePVCs) return;
  uint64_t unb = unbound_of(m, s->lr_objs[self]);
  while (unb) {
    int u = __builtin_ctzll(unb); unb &= unb - 1;
    oval uo = ov_of_u(m, u);
    /* bound == "spec" :> ("pvname" :> unb.n) @@ unb  (:675-676) */
    oval bound = (oval)(uo | (1u << 3));
    kstate t = *s;
    push_api(&t, self, KO_PVCDone);
    t.obj[self] = bound; t.op[self] = OP_Update; t.pc[self] = KO_DoRequest;
    emit(e, &t, 19);
  }
}
static void a_PVCDone(const model *m, const kstate *s, int self, emitter *e) { /* :690-693 */
  (void)m;
  if (s->pc[self] != KO_PVCDone) return;
  kstate t = *s;
  t.pc[self] = KO_PVCStart;
  emit(e, &t, 20);
}
/* APIStart(self)  KubeAPI.tla:698-756 */
static void a_APIStart(const model *m, const kstate *s, int self, emitter *e) {
  if (s->pc[self] != KO_APIStart) return;
  /* \E c \in PendingClients (:699) — processes in index order */
  for (int c = 0; c < m->P; c++) {
    if (!s->rq_present[c] || s->rq_status[c] != ST_Pending) continue;
    kstate t = *s;
    oval o = s->rq_obj[c];
    if (!(o & OV_DEF)) { e->fail_action = 21; e->fail_self = self; return; }
    int id = OV_ID(o);
    uint64_t same = s->api & m->idmask[id];
    switch (s->rq_op[c]) {
    case OP_Create:                                               /* :700-705 */
      br(e, KO_B_API_CREATE);
      if (same) t.rq_status[c] = ST_Error;
      else { t.api |= 1ull << u_of(m, tla_Write(o)); t.rq_status[c] = ST_Ok; }
      break;
    case OP_Force:                                                /* :706-715 */
      br(e, KO_B_API_FORCE);
      /* variant 2 (seeded bug): Force adds the new version without removing
       * the old one, which violates OnlyOneVersion (:787-789) */
      if (same) { br(e, KO_B_API_FORCE_REPLACE);
        t.api = (m->cfg.variant == 2 ? s->api : (s->api & ~same)) | (1ull << u_of(m, tla_Write(o))); }
      else { br(e, KO_B_API_FORCE_CREATE); t.api |= 1ull << u_of(m, tla_Write(o)); }
      t.rq_status[c] = ST_Ok;
      break;
    case OP_Get:                                                  /* :716-728 */
      br(e, KO_B_API_GET);
      if (same) {
        int uc = __builtin_ctzll(same);      /* CHOOSE (unique while OnlyOneVersion) */
        oval chosen = ov_of_u(m, uc);
        t.rq_obj[c] = chosen; t.rq_status[c] = ST_Ok;
        uint64_t nw = s->api & ~same, x = same;
        while (x) {
          int u = __builtin_ctzll(x); x &= x - 1;
          nw |= 1ull << u_of(m, tla_Read(ov_of_u(m, u), c));
        }
        t.api = nw;
      } else { br(e, KO_B_API_GET_NOTFOUND); t.rq_status[c] = ST_Error; }
      break;
    case OP_Delete:                                               /* :729-731 */
      br(e, KO_B_API_DELETE);
      t.api = s->api & ~same; t.rq_status[c] = ST_Ok;
      break;
    case OP_Update: {                                             /* :732-739 */
      br(e, KO_B_API_UPDATE);
      int ok = 0, read = 0;
      uint64_t x = same;
      while (x) {
        int u = __builtin_ctzll(x); x &= x - 1;
        if (tla_HasRead(ov_of_u(m, u), c)) read = 1;
        if (m->cfg.variant == 1 || tla_HasRead(ov_of_u(m, u), c)) ok = 1;
      }
      if (ok) {
        br(e, KO_B_API_UPDATE_OK);
        t.api = (s->api & ~same) | (1ull << u_of(m, tla_Write(o)));
        t.rq_status[c] = ST_Ok;
        /* lostUpdate' = TRUE: the history variable of the build-defined
         * NoLostUpdate (see check_invariants) — an Update applied although
         * its writer read no stored version (possible only in variant 1) */
        if (m->cfg.lost_update && !read) t.api |= KO_LOST_UPDATE;
      } else { br(e, KO_B_API_UPDATE_ERR); t.rq_status[c] = ST_Error; }
      break;
    }
    default:                                                      /* :740-741 */
      br(e, KO_B_API_ASSERT);
      e->fail_action = 21; e->fail_self = self; return;
    }
    emit(e, &t, 21);
  }
  /* \E c \in PendingListClients (:745-753) */
  for (int c = 0; c < m->P; c++) {
    if (!s->lr_present[c] || s->lr_status[c] != ST_Pending) continue;
    br(e, KO_B_API_LIST);
    kstate t = *s;
    int k = s->lr_kind[c];
    uint64_t km = (k == K_Secret) ? m->idmask[ID_SECRET] : (k == K_PVC) ? m->idmask[ID_PVC] : 0;
    /* variant 4 (seeded bug): the reply lists objects of every kind, which
     * violates IsValidListRequest's o.k = r.kind (:435), i.e. TypeOK */
    t.lr_objs[c] = m->cfg.variant == 4 ? (s->api & m->allmask) : (s->api & km);
    t.lr_status[c] = ST_Ok;
    uint64_t nw = s->api & ~km, x = s->api & km;
    while (x) {
      int u = __builtin_ctzll(x); x &= x - 1;
      nw |= 1ull << u_of(m, tla_Read(ov_of_u(m, u), c));
    }
    t.api = nw;
    emit(e, &t, 21);
  }
}

/* Next (KubeAPI.tla:760-763): the action list in TLC's split order. */
static void expand(const model *m, const kstate *s, emitter *e) {
  e->n = 0; e->fail_action = -1; e->fail_self = -1;
  for (int p = 0; p < m->P; p++) {
    a_DoRequest(m, s, p, e);
    a_DoReply(m, s, p, e);
    a_DoListRequest(m, s, p, e);
    a_DoListReply(m, s, p, e);
  }
#define STOP if (e->fail_action >= 0) return
  for (int p = 0; p < m->cfg.nc; p++) {
    a_CStart(m, s, p, e); a_C1(m, s, p, e); a_C10(m, s, p, e); a_C11(m, s, p, e);
    a_c12(m, s, p, e); a_C13(m, s, p, e); a_C2(m, s, p, e); STOP;
    a_C3(m, s, p, e); a_C8(m, s, p, e); a_C6(m, s, p, e); a_C7(m, s, p, e);
    a_C4(m, s, p, e); STOP; a_C5(m, s, p, e);
  }
  for (int p = m->cfg.nc; p < m->cfg.nc + m->cfg.np; p++) {
    a_PVCStart(m, s, p, e); a_PVCListedPVCs(m, s, p, e);
    a_PVCHavePVCs(m, s, p, e); a_PVCDone(m, s, p, e);
  }
  for (int p = m->cfg.nc + m->cfg.np; p < m->P; p++) { a_APIStart(m, s, p, e); STOP; }
#undef STOP
}

/* Init (KubeAPI.tla:455-469); shouldReconcile \in [Clients -> BOOLEAN]
 * enumerated as a binary counter, client 0 least significant, FALSE first. */
static int init_states(const model *m, kstate *out) {
  int n = 1 << m->cfg.nc;
  for (int mask = 0; mask < n; mask++) {
    kstate *t = &out[mask];
    memset(t, 0, sizeof *t);
    for (int p = 0; p < m->P; p++) {
      int k = pkind(m, p);
      t->pc[p] = k == PK_CLIENT ? KO_CStart : k == PK_PVC ? KO_PVCStart : KO_APIStart;
      if (k == PK_CLIENT) t->sr[p] = (mask >> p) & 1;
    }
    /* variant 5 (seeded bug): apiState starts with two versions of
     * Secret/foo (vv {} and vv {process 0}), violating OnlyOneVersion */
    if (m->cfg.variant == 5)
      t->api = (1ull << u_of(m, ov_make(ID_SECRET, 1, 0, 0))) | (1ull << u_of(m, ov_make(ID_SECRET, 1, 0, 1)));
  }
  return n;
}

/* TypeOK (KubeAPI.tla:776-781) and OnlyOneVersion (:787-789).
 * Returns -1 if both hold, else the index of the first violated invariant
 * in MC.cfg order (0 TypeOK, 1 OnlyOneVersion). */
static int check_invariants_all(const model *m, const kstate *s);
/* the invariants the config lists (MC.cfg:13-15); -1 = all hold.
 * NoLostUpdate (index 2, build-defined; SURVEY §8(d) config 5's second
 * variant) == ~lostUpdate, a history variable kept as bit 63 of api (free:
 * apiState has |U| <= 32 bits with at most 3 readers) that APIStart sets
 * when it applies an Update whose writer has not read any stored version of
 * the object (KubeAPI.tla:733 without HasRead: variant 1 only). */
static int check_invariants(const model *m, const kstate *s) {
  int mask = 3 & ~m->cfg.skip_inv, r = -1;
  if (mask) {
    kstate t = *s;
    r = check_invariants_all(m, &t);
    if (r == 0 && !(mask & 1)) {               /* TypeOK fails but is not checked */
      r = -1;
      for (int id = 0; id < 2; id++)
        if (popc64(s->api & m->idmask[id]) > 1) r = (mask & 2) ? 1 : -1;
    } else if (r == 1 && !(mask & 2)) {
      r = -1;
    }
  }
  if (r < 0 && m->cfg.lost_update && (s->api & KO_LOST_UPDATE)) r = 2;
  return r;
}
static int check_invariants_all(const model *m, const kstate *s) {
  int ok = 1;
  /* \A o \in apiState: IsValidAPIObject(o) — every element of U is a record
   * with n,k,vv[,spec] : holds by construction. */
  for (int c = 0; c < m->P && ok; c++) {
    if (s->rq_present[c]) {                              /* IsValidRequest :426-430 */
      if (s->rq_op[c] < OP_Create || s->rq_op[c] > OP_Force) ok = 0;
      if (!(s->rq_obj[c] & OV_DEF)) ok = 0;
      if (s->rq_status[c] < ST_Pending || s->rq_status[c] > ST_Error) ok = 0;
    }
    if (s->lr_present[c]) {                              /* IsValidListRequest :432-436 */
      int k = s->lr_kind[c];
      uint64_t km = (k == K_Secret) ? m->idmask[ID_SECRET] : (k == K_PVC) ? m->idmask[ID_PVC] : 0;
      if (s->lr_objs[c] & ~km) ok = 0;
      if (s->lr_status[c] < ST_Pending || s->lr_status[c] > ST_Error) ok = 0;
    }
  }
  if (!ok) return 0;
  for (int id = 0; id < 2; id++)
    if (popc64(s->api & m->idmask[id]) > 1) return 1;
  return -1;
}


/* --------------------------------------------------------- fingerprints */
static inline uint64_t mix64(uint64_t z) {
  z ^= z >> 30; z *= 0xbf58476d1ce4e5b9ull;
  z ^= z >> 27; z *= 0x94d049bb133111ebull;
  z ^= z >> 31; return z;
}
static inline void fp128(const kstate *s, uint64_t *h1, uint64_t *h2) {
  const uint64_t *w = (const uint64_t *)s;
  uint64_t a = 0x243f6a8885a308d3ull, b = 0x13198a2e03707344ull;
  for (size_t i = 0; i < sizeof(kstate) / 8; i++) {
    a = mix64(a ^ w[i]) + 0x9e3779b97f4a7c15ull;
    b = (b ^ w[i]) * 0xff51afd7ed558ccdull; b ^= b >> 33;
  }
  a = mix64(a); b = mix64(b ^ 0xc4ceb9fe1a85ec53ull);
  if (a == 0) a = 1;
  *h1 = a; *h2 = b;
}

/* Seen-set of fingerprints.  wide=1: 128-bit entries (default, exact for
 * all practical purposes); wide=0: 64-bit entries (TLC-like; used for the
 * largest runs where 128-bit entries would not fit in host RAM). */
typedef struct { uint64_t *slots; uint64_t mask, count; int wide, fixed; } fpset128;
static void fs_init2(fpset128 *f, uint64_t cap_pow2, int wide, int fixed) {
  f->slots = calloc((wide ? 2 : 1) * cap_pow2, sizeof(uint64_t));
  if (!f->slots) { fprintf(stderr, "kubeapi_oracle: out of memory\n"); abort(); }
  f->mask = cap_pow2 - 1; f->count = 0; f->wide = wide; f->fixed = fixed;
}
static void fs_init(fpset128 *f, uint64_t cap_pow2) { fs_init2(f, cap_pow2, 1, 0); }
static int fs_put_raw(fpset128 *f, uint64_t a, uint64_t b) { /* 1 if new */
  uint64_t i = (a * 0x9e3779b97f4a7c15ull >> 17) & f->mask;
  if (!f->wide) {
    for (;;) {
      uint64_t *sl = &f->slots[i];
      if (*sl == 0) { *sl = a; f->count++; return 1; }
      if (*sl == a) return 0;
      i = (i + 1) & f->mask;
    }
  }
  for (;;) {
    uint64_t *sl = &f->slots[2 * i];
    if (sl[0] == 0) { sl[0] = a; sl[1] = b; f->count++; return 1; }
    if (sl[0] == a && sl[1] == b) return 0;
    i = (i + 1) & f->mask;
  }
}
static int fs_put(fpset128 *f, uint64_t a, uint64_t b) {
  if ((f->count + 1) * 4 > (f->mask + 1) * 3 && f->fixed) {
    fprintf(stderr, "kubeapi_oracle: presized fpset full\n"); abort();
  }
  if (!f->fixed && (f->count + 1) * 2 > f->mask + 1) {   /* grow at 50% load */
    fpset128 g; fs_init2(&g, 2 * (f->mask + 1), f->wide, 0);
    for (uint64_t i = 0; i <= f->mask; i++) {
      if (f->wide) { if (f->slots[2 * i]) fs_put_raw(&g, f->slots[2 * i], f->slots[2 * i + 1]); }
      else if (f->slots[i]) fs_put_raw(&g, f->slots[i], 0);
    }
    free(f->slots); *f = g;
  }
  return fs_put_raw(f, a, b);
}

/* ---------------------------------------------------------------- names */
static const char *ACTION_NAMES[KO_NACTIONS] = {
  "DoRequest", "DoReply", "DoListRequest", "DoListReply", "CStart", "C1", "C10",
  "C11", "c12", "C13", "C2", "C3", "C8", "C6", "C7", "C4", "C5", "PVCStart",
  "PVCListedPVCs", "PVCHavePVCs", "PVCDone", "APIStart"};
const char *ko_action_name(int a) { return (a >= 0 && a < KO_NACTIONS) ? ACTION_NAMES[a] : "?"; }
static const char *LABELS[KO_NPC] = {
  "?", "CStart", "C1", "C10", "C11", "c12", "C13", "C2", "C3", "C8", "C6", "C7",
  "C4", "C5", "PVCStart", "PVCListedPVCs", "PVCHavePVCs", "PVCDone", "APIStart",
  "DoRequest", "DoReply", "DoListRequest", "DoListReply"};
const char *ko_label_name(int pc) { return (pc >= 0 && pc < KO_NPC) ? LABELS[pc] : "?"; }

/* ------------------------------------------------------------ canonical */
int ko_tuple_words(const ko_config *cfg) {
  return 1 + KO_TUPLE_PER_PROC * (cfg->nc + cfg->np + cfg->ns);
}
static void to_tuple(const model *m, const kstate *s, uint64_t *o) {
  int k = 0;
  o[k++] = s->api;
  for (int p = 0; p < m->P; p++) {
    o[k++] = s->pc[p]; o[k++] = s->op[p]; o[k++] = s->obj[p]; o[k++] = s->kind[p];
    o[k++] = s->sr[p]; o[k++] = s->sdepth[p]; o[k++] = s->sproc[p]; o[k++] = s->spc[p];
    o[k++] = s->sop[p]; o[k++] = s->sobj[p]; o[k++] = s->skind[p];
    o[k++] = s->rq_present[p]; o[k++] = s->rq_op[p]; o[k++] = s->rq_status[p];
    o[k++] = s->rq_obj[p];
    o[k++] = s->lr_present[p]; o[k++] = s->lr_kind[p]; o[k++] = s->lr_status[p];
    o[k++] = s->lr_objs[p];
  }
}
static void from_tuple(const model *m, const uint64_t *o, kstate *s) {
  memset(s, 0, sizeof *s);
  int k = 0;
  s->api = o[k++];
  for (int p = 0; p < m->P; p++) {
    s->pc[p] = (uint8_t)o[k++]; s->op[p] = (uint8_t)o[k++]; s->obj[p] = (uint8_t)o[k++];
    s->kind[p] = (uint8_t)o[k++]; s->sr[p] = (uint8_t)o[k++]; s->sdepth[p] = (uint8_t)o[k++];
    s->sproc[p] = (uint8_t)o[k++]; s->spc[p] = (uint8_t)o[k++]; s->sop[p] = (uint8_t)o[k++];
    s->sobj[p] = (uint8_t)o[k++]; s->skind[p] = (uint8_t)o[k++];
    s->rq_present[p] = (uint8_t)o[k++]; s->rq_op[p] = (uint8_t)o[k++];
    s->rq_status[p] = (uint8_t)o[k++]; s->rq_obj[p] = (uint8_t)o[k++];
    s->lr_present[p] = (uint8_t)o[k++]; s->lr_kind[p] = (uint8_t)o[k++];
    s->lr_status[p] = (uint8_t)o[k++]; s->lr_objs[p] = o[k++];
  }
}

/* Compact storage form for frontiers: api, then per process one word of
 * scalar fields and one word of listRequests[p].objs (72 B at P=4). */
#define PACKW (1 + 2 * KO_MAXP)
typedef struct { uint64_t w[PACKW]; } kpacked;
static void kpack(const model *m, const kstate *s, kpacked *o) {
  memset(o, 0, sizeof *o);
  o->w[0] = s->api;
  for (int p = 0; p < m->P; p++) {
    uint64_t x = 0; int b = 0;
#define PUT(v, n) do { x |= (uint64_t)(v) << b; b += (n); } while (0)
    PUT(s->pc[p], 5); PUT(s->op[p], 3); PUT(s->obj[p], 8); PUT(s->kind[p], 2);
    PUT(s->sr[p], 1); PUT(s->sdepth[p], 1); PUT(s->sproc[p], 2); PUT(s->spc[p], 5);
    PUT(s->sop[p], 3); PUT(s->sobj[p], 8); PUT(s->skind[p], 2); PUT(s->rq_present[p], 1);
    PUT(s->rq_op[p], 3); PUT(s->rq_status[p], 2); PUT(s->rq_obj[p], 8);
    PUT(s->lr_present[p], 1); PUT(s->lr_kind[p], 2); PUT(s->lr_status[p], 2);
#undef PUT
    o->w[1 + 2 * p] = x; o->w[2 + 2 * p] = s->lr_objs[p];
  }
}
static void kunpack(const model *m, const kpacked *o, kstate *s) {
  memset(s, 0, sizeof *s);
  s->api = o->w[0];
  for (int p = 0; p < m->P; p++) {
    uint64_t x = o->w[1 + 2 * p]; int b = 0;
#define GET(f, n) do { f = (uint8_t)((x >> b) & ((1u << (n)) - 1)); b += (n); } while (0)
    GET(s->pc[p], 5); GET(s->op[p], 3); GET(s->obj[p], 8); GET(s->kind[p], 2);
    GET(s->sr[p], 1); GET(s->sdepth[p], 1); GET(s->sproc[p], 2); GET(s->spc[p], 5);
    GET(s->sop[p], 3); GET(s->sobj[p], 8); GET(s->skind[p], 2); GET(s->rq_present[p], 1);
    GET(s->rq_op[p], 3); GET(s->rq_status[p], 2); GET(s->rq_obj[p], 8);
    GET(s->lr_present[p], 1); GET(s->lr_kind[p], 2); GET(s->lr_status[p], 2);
#undef GET
    s->lr_objs[p] = o->w[2 + 2 * p];
  }
}

/* ------------------------------------------------------------- printing */
static const char *pname(const model *m, int p, char *buf) {
  int k = pkind(m, p);
  const char *base = k == PK_CLIENT ? "Client" : k == PK_PVC ? "PVCController" : "Server";
  int cnt = k == PK_CLIENT ? m->cfg.nc : k == PK_PVC ? m->cfg.np : m->cfg.ns;
  int idx = k == PK_CLIENT ? p : k == PK_PVC ? p - m->cfg.nc : p - m->cfg.nc - m->cfg.np;
  if (cnt == 1) snprintf(buf, 32, "%s", base); else snprintf(buf, 32, "%s%d", base, idx + 1);
  return buf;
}
typedef struct { char *buf; size_t cap, len; } sbuf;
static void sb_put(sbuf *b, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
#include <stdarg.h>
static void sb_put(sbuf *b, const char *fmt, ...) {
  char tmp[512]; va_list ap; va_start(ap, fmt);
  int n = vsnprintf(tmp, sizeof tmp, fmt, ap); va_end(ap);
  if (b->buf && b->len + n < b->cap) memcpy(b->buf + b->len, tmp, n + 1);
  b->len += n;
}
static void put_set_procs(const model *m, sbuf *b, int vv) {
  char nb[32]; int first = 1;
  sb_put(b, "{");
  for (int c = 0; c < m->R; c++) if ((vv >> c) & 1) { sb_put(b, "%s\"%s\"", first ? "" : ", ", pname(m, c, nb)); first = 0; }
  sb_put(b, "}");
}
static void put_oval(const model *m, sbuf *b, oval o) {
  if (!(o & OV_DEF)) { sb_put(b, "defaultInitValue"); return; }
  int id = OV_ID(o);
  sb_put(b, "[k |-> \"%s\", n |-> \"%s\"", id == ID_SECRET ? "Secret" : "PVC", id == ID_SECRET ? "foo" : "mypvc");
  if (OV_SPEC(o)) sb_put(b, ", spec |-> [pvname |-> \"%s\"]", id == ID_SECRET ? "foo" : "mypvc");
  if (OV_HASVV(o)) { sb_put(b, ", vv |-> "); put_set_procs(m, b, OV_VV(o)); }
  sb_put(b, "]");
}
static void put_uset(const model *m, sbuf *b, uint64_t set) {
  sb_put(b, "{"); int first = 1;
  while (set) { int u = __builtin_ctzll(set); set &= set - 1;
    if (!first) { sb_put(b, ", "); } first = 0; put_oval(m, b, ov_of_u(m, u)); }
  sb_put(b, "}");
}
static const char *OPN[] = {"defaultInitValue", "\"Create\"", "\"Get\"", "\"Update\"", "\"Delete\"", "\"Force\""};
static const char *STN[] = {"?", "\"Pending\"", "\"Ok\"", "\"Error\""};
static const char *KN[] = {"defaultInitValue", "\"Secret\"", "\"PVC\""};
static void put_state(const model *m, sbuf *b, const kstate *s) {
  char nb[32]; int first;
  sb_put(b, "/\\ apiState = "); put_uset(m, b, s->api & m->allmask);
  sb_put(b, "\n/\\ requests = "); first = 1;
  for (int c = 0; c < m->P; c++) if (s->rq_present[c]) {
    sb_put(b, "%s\"%s\" :> [op |-> %s, obj |-> ", first ? "(" : " @@ ", pname(m, c, nb), OPN[s->rq_op[c]]);
    put_oval(m, b, s->rq_obj[c]); sb_put(b, ", status |-> %s]", STN[s->rq_status[c]]); first = 0; }
  sb_put(b, first ? "<<>>" : ")");
  sb_put(b, "\n/\\ listRequests = "); first = 1;
  for (int c = 0; c < m->P; c++) if (s->lr_present[c]) {
    sb_put(b, "%s\"%s\" :> [kind |-> %s, objs |-> ", first ? "(" : " @@ ", pname(m, c, nb), KN[s->lr_kind[c]]);
    put_uset(m, b, s->lr_objs[c]); sb_put(b, ", status |-> %s]", STN[s->lr_status[c]]); first = 0; }
  sb_put(b, first ? "<<>>" : ")");
  sb_put(b, "\n/\\ pc = ("); for (int p = 0; p < m->P; p++) sb_put(b, "%s\"%s\" :> \"%s\"", p ? " @@ " : "", pname(m, p, nb), LABELS[s->pc[p]]);
  sb_put(b, ")\n/\\ stack = (");
  for (int p = 0; p < m->P; p++) {
    sb_put(b, "%s\"%s\" :> ", p ? " @@ " : "", pname(m, p, nb));
    if (!s->sdepth[p]) sb_put(b, "<<>>");
    else if (s->sproc[p] == PR_API) { sb_put(b, "<<[procedure |-> \"API\", pc |-> \"%s\", op |-> %s, obj |-> ", LABELS[s->spc[p]], OPN[s->sop[p]]); put_oval(m, b, s->sobj[p]); sb_put(b, "]>>"); }
    else sb_put(b, "<<[procedure |-> \"ListAPI\", pc |-> \"%s\", kind |-> %s]>>", LABELS[s->spc[p]], KN[s->skind[p]]);
  }
  sb_put(b, ")\n/\\ op = ("); for (int p = 0; p < m->P; p++) sb_put(b, "%s\"%s\" :> %s", p ? " @@ " : "", pname(m, p, nb), OPN[s->op[p]]);
  sb_put(b, ")\n/\\ obj = ("); for (int p = 0; p < m->P; p++) { sb_put(b, "%s\"%s\" :> ", p ? " @@ " : "", pname(m, p, nb)); put_oval(m, b, s->obj[p]); }
  sb_put(b, ")\n/\\ kind = ("); for (int p = 0; p < m->P; p++) sb_put(b, "%s\"%s\" :> %s", p ? " @@ " : "", pname(m, p, nb), KN[s->kind[p]]);
  sb_put(b, ")\n/\\ shouldReconcile = (");
  for (int p = 0; p < m->cfg.nc; p++) sb_put(b, "%s\"%s\" :> %s", p ? " @@ " : "", pname(m, p, nb), s->sr[p] ? "TRUE" : "FALSE");
  sb_put(b, ")\n");
  if (m->cfg.lost_update) sb_put(b, "/\\ lostUpdate = %s\n", (s->api & KO_LOST_UPDATE) ? "TRUE" : "FALSE");
}

/* ------------------------------------------------------------------ BFS */
typedef struct {
  model m;
  kstate *trace; int trace_len;
  char msg[256];
} handle_t;

typedef struct { kstate *v; uint64_t n, cap; } svec;
static void sv_push(svec *a, const kstate *s) {
  if (a->n == a->cap) { a->cap = a->cap ? a->cap * 2 : 1024; a->v = realloc(a->v, a->cap * sizeof(kstate));
    if (!a->v) { fprintf(stderr, "kubeapi_oracle: out of memory\n"); abort(); } }
  a->v[a->n++] = *s;
}
typedef struct { uint64_t *v; uint64_t n, cap; int words; } pvec;  /* packed states */
static void pv_push(pvec *a, const model *m, const kstate *s) {
  if (a->n == a->cap) { a->cap = a->cap ? a->cap * 2 : 1024;
    a->v = realloc(a->v, a->cap * a->words * 8);
    if (!a->v) { fprintf(stderr, "kubeapi_oracle: out of memory\n"); abort(); } }
  kpacked k; kpack(m, s, &k);
  memcpy(a->v + a->n * a->words, k.w, a->words * 8); a->n++;
}
static void pv_get(const pvec *a, const model *m, uint64_t i, kstate *s) {
  kpacked k; memset(&k, 0, sizeof k); memcpy(k.w, a->v + i * a->words, a->words * 8);
  kunpack(m, &k, s);
}
typedef struct { uint64_t *parent; uint16_t *ord; uint64_t n, cap; } tvec;
static void tv_push(tvec *t, uint64_t parent, int ord) {
  if (t->n == t->cap) { t->cap = t->cap ? t->cap * 2 : 4096;
    t->parent = realloc(t->parent, t->cap * 8); t->ord = realloc(t->ord, t->cap * 2);
    if (!t->parent || !t->ord) { fprintf(stderr, "kubeapi_oracle: out of memory\n"); abort(); } }
  t->parent[t->n] = parent; t->ord[t->n] = (uint16_t)ord; t->n++;
}

#define MAXSUCC 64
static void rebuild_trace(handle_t *h, const tvec *tv, uint64_t last_gidx, const kstate *inits) {
  int len = 0; uint64_t g = last_gidx;
  for (;;) { len++; if (tv->parent[g] == UINT64_MAX) break; g = tv->parent[g]; }
  uint64_t *chain = malloc(len * 8);
  g = last_gidx;
  for (int i = len - 1; i >= 0; i--) { chain[i] = g; g = tv->parent[g]; }
  h->trace = malloc(len * sizeof(kstate)); h->trace_len = len;
  h->trace[0] = inits[tv->ord[chain[0]]];
  kstate succ[MAXSUCC]; uint8_t act[MAXSUCC];
  emitter e = {succ, act, 0, MAXSUCC, -1, -1, NULL};
  for (int i = 1; i < len; i++) {
    expand(&h->m, &h->trace[i - 1], &e);
    h->trace[i] = succ[tv->ord[chain[i]]];
  }
  free(chain);
}

void *ko_run(const ko_config *cfg, ko_result *res) {
  handle_t *h = calloc(1, sizeof *h);
  model_init(&h->m, cfg);
  const model *m = &h->m;
  memset(res, 0, sizeof *res);
  res->err_action = res->err_self = res->err_invariant = -1;
  struct timespec t0, t1; clock_gettime(CLOCK_MONOTONIC, &t0);

  fpset128 fs;
  if (cfg->fpset_log2 > 0) fs_init2(&fs, 1ull << cfg->fpset_log2, cfg->fp_bits != 64, 1);
  else fs_init2(&fs, 1 << 16, cfg->fp_bits != 64, 0);
  int pw = 1 + 2 * (cfg->nc + cfg->np + cfg->ns);
  pvec cur = {0, 0, 0, pw}, nxt = {0, 0, 0, pw};
  kstate scur;
  tvec tv = {0};
  uint64_t cur_base = 0;  /* gidx of cur.v[0] */
  kstate inits[1 << 4];
  int ni = init_states(m, inits);
  uint64_t branch[NBRANCH] = {0};
  uint64_t fail_gidx = UINT64_MAX;

  for (int i = 0; i < ni; i++) {
    uint64_t a, b; fp128(&inits[i], &a, &b);
    res->generated++;
    if (fs_put(&fs, a, b)) {
      pv_push(&cur, m, &inits[i]);
      if (cfg->keep_trace) tv_push(&tv, UINT64_MAX, i);
      int inv = check_invariants(m, &inits[i]);
      if (inv >= 0 && !res->err_kind) { res->err_kind = KO_ERR_INVARIANT; res->err_invariant = inv;
        fail_gidx = cur.n - 1; res->err_level = 1; }
    }
  }
  res->init = cur.n;
  res->distinct = cur.n;
  kstate succ[MAXSUCC]; uint8_t act[MAXSUCC];
  emitter e = {succ, act, 0, MAXSUCC, -1, -1, branch};
  int level = 1;
  while (cur.n > 0 && !res->err_kind) {
    if (level > KO_MAXLEVELS - 1) break;
    res->level_width[level - 1] = cur.n;
    res->nlevels = level;
    if (cfg->max_levels && level >= cfg->max_levels) break;
    nxt.n = 0;
    for (uint64_t i = 0; i < cur.n && !res->err_kind; i++) {
      pv_get(&cur, m, i, &scur);
      const kstate *s = &scur;
      /* per-distinct-state coverage sums (MC.out:1029-1080) */
      int na = popc64(s->api & m->allmask);
      res->cov_api += na; res->cov_api2 += (uint64_t)na * na;
      for (int c = 0; c < m->P; c++) {
        res->cov_req += s->rq_present[c];
        if (s->lr_present[c]) { res->cov_lreq++; res->cov_objs += popc64(s->lr_objs[c]); }
      }
      expand(m, s, &e);
      int fresh = 0;
      /* successors generated before a failing action are still generated */
      for (int k = 0; k < e.n; k++) {
        res->generated++; res->act_gen[act[k]]++;
        uint64_t a, b; fp128(&succ[k], &a, &b);
        if (fs_put(&fs, a, b)) {
          fresh++;
          res->act_dist[act[k]]++;
          pv_push(&nxt, m, &succ[k]);
          if (cfg->keep_trace) tv_push(&tv, cur_base + i, k);
          int inv = check_invariants(m, &succ[k]);
          if (inv >= 0) { res->err_kind = KO_ERR_INVARIANT; res->err_invariant = inv;
            fail_gidx = cur_base + cur.n + nxt.n - 1; res->err_level = level + 1; break; }
        }
      }
      if (res->err_kind) break;
      if (e.fail_action >= 0) {
        res->err_kind = KO_ERR_ASSERT; res->err_action = e.fail_action; res->err_self = e.fail_self;
        fail_gidx = cur_base + i; res->err_level = level; break;
      }
      res->outdeg_hist[e.n < 31 ? e.n : 31]++;
      res->newdeg_hist[fresh < 31 ? fresh : 31]++;
      if (e.n == 0 && cfg->check_deadlock) {
        res->err_kind = KO_ERR_DEADLOCK; fail_gidx = cur_base + i; res->err_level = level; break;
      }
    }
    res->distinct += nxt.n;
    cur_base += cur.n;
    pvec tmp = cur; cur = nxt; nxt = tmp;
    level++;
    if (cfg->progress) fprintf(stderr, "level %d: width %llu distinct %llu generated %llu\n",
                               level - 1, (unsigned long long)cur.n, (unsigned long long)res->distinct,
                               (unsigned long long)res->generated);
    if (cfg->max_distinct && res->distinct >= cfg->max_distinct) break;
  }
  res->depth = res->nlevels;
  res->queue_left = res->err_kind ? 0 : cur.n;
  res->complete = (cur.n == 0 && !res->err_kind);
  memcpy(res->branch, branch, sizeof branch);
  if (res->err_kind && cfg->keep_trace && fail_gidx != UINT64_MAX) {
    rebuild_trace(h, &tv, fail_gidx, inits);
    res->trace_len = h->trace_len;
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  res->seconds = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
  free(fs.slots); free(cur.v); free(nxt.v); free(tv.parent); free(tv.ord);
  return h;
}

size_t ko_trace_text(void *hv, char *buf, size_t cap) {
  handle_t *h = hv;
  sbuf b = {buf, cap, 0};
  if (buf && cap) buf[0] = 0;
  if (!h) return 0;
  for (int i = 0; i < h->trace_len; i++) {
    sb_put(&b, "State %d:\n", i + 1);
    put_state(&h->m, &b, &h->trace[i]);
    sb_put(&b, "\n");
  }
  return b.len + 1;
}
int ko_trace_tuple(void *hv, int i, uint64_t *out) {
  handle_t *h = hv;
  if (!h || i < 0 || i >= h->trace_len) return 0;
  to_tuple(&h->m, &h->trace[i], out);
  return ko_tuple_words(&h->m.cfg);
}
void ko_free(void *hv) {
  handle_t *h = hv;
  if (!h) return;
  free(h->trace); free(h);
}

uint64_t ko_level_tuples(const ko_config *cfg, int level, uint64_t *out, uint64_t cap_states) {
  model m; model_init(&m, cfg);
  fpset128 fs; fs_init(&fs, 1 << 16);
  svec cur = {0}, nxt = {0};
  kstate inits[16]; int ni = init_states(&m, inits);
  for (int i = 0; i < ni; i++) { uint64_t a, b; fp128(&inits[i], &a, &b); if (fs_put(&fs, a, b)) sv_push(&cur, &inits[i]); }
  kstate succ[MAXSUCC]; uint8_t act[MAXSUCC];
  emitter e = {succ, act, 0, MAXSUCC, -1, -1, NULL};
  for (int l = 1; l < level && cur.n; l++) {
    nxt.n = 0;
    for (uint64_t i = 0; i < cur.n; i++) {
      expand(&m, &cur.v[i], &e);
      for (int k = 0; k < e.n; k++) { uint64_t a, b; fp128(&succ[k], &a, &b); if (fs_put(&fs, a, b)) sv_push(&nxt, &succ[k]); }
    }
    svec t = cur; cur = nxt; nxt = t;
  }
  uint64_t n = cur.n;
  if (out) {
    int w = ko_tuple_words(cfg);
    for (uint64_t i = 0; i < n && i < cap_states; i++) to_tuple(&m, &cur.v[i], out + i * w);
  }
  free(fs.slots); free(cur.v); free(nxt.v);
  return n;
}

int ko_successors(const ko_config *cfg, const uint64_t *tuple, int *actions,
                  uint64_t *succ_tuples, int cap, int *fail_action) {
  model m; model_init(&m, cfg);
  kstate s; from_tuple(&m, tuple, &s);
  kstate succ[MAXSUCC]; uint8_t act[MAXSUCC];
  emitter e = {succ, act, 0, MAXSUCC, -1, -1, NULL};
  expand(&m, &s, &e);
  if (fail_action) *fail_action = e.fail_action;
  int w = ko_tuple_words(cfg);
  for (int k = 0; k < e.n && k < cap; k++) {
    if (actions) actions[k] = act[k];
    if (succ_tuples) to_tuple(&m, &succ[k], succ_tuples + (size_t)k * w);
  }
  return e.fail_action >= 0 ? -1 : e.n;
}

double ko_bench_sample(const ko_config *cfg, double budget, uint64_t *states_done) {
  /* Full BFS from Init, timing everything, stopped once `budget` seconds of
   * work have elapsed (checked per level).  Returns distinct states/s. */
  model m; model_init(&m, cfg);
  struct timespec t0, t1; clock_gettime(CLOCK_MONOTONIC, &t0);
  fpset128 fs; fs_init(&fs, 1 << 20);
  svec cur = {0}, nxt = {0};
  kstate inits[16]; int ni = init_states(&m, inits);
  uint64_t distinct = 0;
  for (int i = 0; i < ni; i++) { uint64_t a, b; fp128(&inits[i], &a, &b); if (fs_put(&fs, a, b)) { sv_push(&cur, &inits[i]); distinct++; } }
  kstate succ[MAXSUCC]; uint8_t act[MAXSUCC];
  emitter e = {succ, act, 0, MAXSUCC, -1, -1, NULL};
  double el = 0;
  while (cur.n) {
    nxt.n = 0;
    for (uint64_t i = 0; i < cur.n; i++) {
      expand(&m, &cur.v[i], &e);
      for (int k = 0; k < e.n; k++) { uint64_t a, b; fp128(&succ[k], &a, &b); if (fs_put(&fs, a, b)) sv_push(&nxt, &succ[k]); }
      if ((i & 4095) == 0) {
        clock_gettime(CLOCK_MONOTONIC, &t1);
        el = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
        if (el > budget) { distinct += nxt.n; goto done; }
      }
    }
    distinct += nxt.n;
    svec t = cur; cur = nxt; nxt = t;
  }
done:
  clock_gettime(CLOCK_MONOTONIC, &t1);
  el = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
  free(fs.slots); free(cur.v); free(nxt.v);
  if (states_done) *states_done = distinct;
  return el > 0 ? distinct / el : 0;
}

/* ------------------------------------------------ multi-core comparator */
/* A level-synchronous BFS of the same spec on `threads` host threads: the
 * CPU comparator bench.py times next to the GPU (TLC's "-workers = all host
 * cores" role; the reference run used 4 workers, MC.out:5).
 * A persistent pool of threads (one barrier per level) takes chunks of the
 * frontier, expands them with the same action functions as ko_run, and
 * inserts 64-bit fingerprints into one lock-free open-addressing set (CAS
 * on the slot; the table is transparent-huge-page backed); new states go to
 * the thread's own next-frontier buffer, concatenated after the level.
 * Counts (distinct, generated, level widths) equal ko_run's; which parent
 * first reaches a state depends on thread timing, so per-action distinct
 * splits are not reproduced (they are not reported).  Stops after `budget`
 * seconds (checked every chunk) or at the end of the state space. */
#include <pthread.h>
#include <stdatomic.h>
#include <sys/mman.h>

typedef struct {
  const model *m;
  pvec cur;
  _Atomic uint64_t next;            /* next frontier index to take */
  _Atomic uint64_t *slots;          /* fingerprint set (0 = empty) */
  unsigned __int128 *slots2;        /* or (fp_bits 128) two-hash keys (0 = empty) */
  uint64_t mask;
  struct timespec t0;
  double budget;
  _Atomic int stop;
  int done;                         /* the pool exits */
  pthread_barrier_t start, end;
} par_level;

typedef struct {
  par_level *L;
  pvec out;
  uint64_t generated;
} par_worker;

static double elapsed_since(const struct timespec *t0) {
  struct timespec t1; clock_gettime(CLOCK_MONOTONIC, &t1);
  return (t1.tv_sec - t0->tv_sec) + 1e-9 * (t1.tv_nsec - t0->tv_nsec);
}

static void pv_append(pvec *a, const uint64_t *w) {
  if (a->n == a->cap) { a->cap = a->cap ? a->cap * 2 : 4096;
    a->v = realloc(a->v, a->cap * a->words * 8);
    if (!a->v) { fprintf(stderr, "kubeapi_oracle: out of memory\n"); abort(); } }
  memcpy(a->v + a->n * a->words, w, a->words * 8); a->n++;
}
/* 64-bit fingerprint of packed canonical words (nonzero) */
static uint64_t packed_fp(const uint64_t *w, int n) {
  uint64_t a = 0x243f6a8885a308d3ull;
  for (int i = 0; i < n; i++) a = mix64(a ^ w[i]) + 0x9e3779b97f4a7c15ull;
  return a ? a : 1;
}

/* a second, independent 64-bit hash of the same words (128-bit keys) */
static uint64_t packed_fp2(const uint64_t *w, int n) {
  uint64_t a = 0x13198a2e03707344ull;
  for (int i = 0; i < n; i++) a = mix64((a + 0xa4093822299f31d0ull) ^ (w[i] * 0xff51afd7ed558ccdull));
  return a ? a : 1;
}
/* 128-bit keys: every probe is one locked 16-byte compare-exchange (the
 * returned value is the slot's, read atomically), so no torn read of a
 * slot being filled can look like another key */
static int par_insert2(par_level *L, uint64_t h1, uint64_t h2) {   /* 1 if new */
  const unsigned __int128 key = ((unsigned __int128)h2 << 64) | h1;
  uint64_t i = (h1 * 0x9e3779b97f4a7c15ull >> 17) & L->mask;
  for (;;) {
    const unsigned __int128 e = __sync_val_compare_and_swap(&L->slots2[i], (unsigned __int128)0, key);
    if (e == 0) return 1;
    if (e == key) return 0;
    i = (i + 1) & L->mask;
  }
}

static int par_insert(par_level *L, uint64_t fp) {   /* 1 if new */
  if (!fp) fp = 1;
  uint64_t i = (fp * 0x9e3779b97f4a7c15ull >> 17) & L->mask;
  for (;;) {
    uint64_t e = atomic_load_explicit(&L->slots[i], memory_order_relaxed);
    if (e == fp) return 0;
    if (e == 0) {
      uint64_t z = 0;
      if (atomic_compare_exchange_strong(&L->slots[i], &z, fp)) return 1;
      if (z == fp) return 0;
    }
    i = (i + 1) & L->mask;
  }
}

static void *par_work(void *arg) {
  par_worker *w = arg;
  par_level *L = w->L;
  const model *m = L->m;
  kstate s, succ[MAXSUCC]; uint8_t act[MAXSUCC];
  emitter e = {succ, act, 0, MAXSUCC, -1, -1, NULL};
  const int pw = L->cur.words;
  for (;;) {
    pthread_barrier_wait(&L->start);
    if (L->done) break;
    for (;;) {
      if (atomic_load_explicit(&L->stop, memory_order_relaxed)) break;
      uint64_t i0 = atomic_fetch_add(&L->next, 512);
      if (i0 >= L->cur.n) break;
      uint64_t i1 = i0 + 512 < L->cur.n ? i0 + 512 : L->cur.n;
      for (uint64_t i = i0; i < i1; i++) {
        pv_get(&L->cur, m, i, &s);
        expand(m, &s, &e);
        for (int k = 0; k < e.n; k++) {
          w->generated++;
          /* the packed words are canonical: hash those (cheaper than the
           * whole kstate) and store them as they are */
          kpacked pk; kpack(m, &succ[k], &pk);
          const int fresh = L->slots2 ? par_insert2(L, packed_fp(pk.w, pw), packed_fp2(pk.w, pw))
                                      : par_insert(L, packed_fp(pk.w, pw));
          if (fresh) pv_append(&w->out, pk.w);
        }
      }
      if (elapsed_since(&L->t0) > L->budget) atomic_store(&L->stop, 1);
    }
    pthread_barrier_wait(&L->end);
  }
  return NULL;
}

double ko_bench_parallel(const ko_config *cfg, int threads, double budget, ko_par_result *out) {
  model m; model_init(&m, cfg);
  memset(out, 0, sizeof *out);
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  const int log2 = cfg->fpset_log2 > 0 ? cfg->fpset_log2 : 28;
  const int wide = cfg->fp_bits == 128;       /* (explicit: the timed comparator keeps 64-bit keys) */
  static par_level L;
  memset(&L, 0, sizeof L);
  L.m = &m; L.mask = (1ull << log2) - 1; L.budget = budget;
  const size_t bytes = (1ull << log2) * (wide ? 16 : sizeof(uint64_t));
  clock_gettime(CLOCK_MONOTONIC, &L.t0);
  void *mem = mmap(NULL, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (mem == MAP_FAILED) { fprintf(stderr, "kubeapi_oracle: out of memory\n"); abort(); }
  madvise(mem, bytes, MADV_HUGEPAGE);
  if (wide) L.slots2 = mem; else L.slots = mem;
  out->fp_bits = wide ? 128 : 64;
  const int pw = 1 + 2 * (cfg->nc + cfg->np + cfg->ns);
  L.cur = (pvec){0, 0, 0, pw};
  kstate inits[16]; int ni = init_states(&m, inits);
  for (int i = 0; i < ni; i++) {
    kpacked pk; kpack(&m, &inits[i], &pk);
    out->generated++;
    const int fresh = wide ? par_insert2(&L, packed_fp(pk.w, pw), packed_fp2(pk.w, pw))
                           : par_insert(&L, packed_fp(pk.w, pw));
    if (fresh) pv_append(&L.cur, pk.w);
  }
  out->distinct = L.cur.n;
  out->depth = 1;
  out->level_width[0] = L.cur.n;
  par_worker *W = calloc(threads, sizeof *W);
  pthread_t *T = calloc(threads, sizeof *T);
  pthread_barrier_init(&L.start, NULL, threads + 1);
  pthread_barrier_init(&L.end, NULL, threads + 1);
  for (int t = 0; t < threads; t++) {
    W[t].L = &L; W[t].out.words = pw;
    pthread_create(&T[t], NULL, par_work, &W[t]);
  }
  while (L.cur.n && !atomic_load(&L.stop)) {
    if (cfg->max_levels && out->depth >= cfg->max_levels) break;   /* (as the engine: depth max_levels) */
    out->levels++;
    atomic_store(&L.next, 0);
    for (int t = 0; t < threads; t++) W[t].out.n = 0;
    pthread_barrier_wait(&L.start);
    pthread_barrier_wait(&L.end);
    uint64_t total = 0;
    for (int t = 0; t < threads; t++) {
      total += W[t].out.n;
      out->generated += W[t].generated;
      W[t].generated = 0;
    }
    pvec nxt = {0, 0, 0, pw};
    nxt.cap = total ? total : 1;
    nxt.v = malloc(nxt.cap * pw * 8);
    if (!nxt.v) { fprintf(stderr, "kubeapi_oracle: out of memory\n"); abort(); }
    for (int t = 0; t < threads; t++) {
      memcpy(nxt.v + nxt.n * pw, W[t].out.v, W[t].out.n * pw * 8);
      nxt.n += W[t].out.n;
    }
    out->distinct += total;
    if (total && out->depth < KO_MAXLEVELS) out->level_width[out->depth++] = total;
    free(L.cur.v);
    L.cur = nxt;
    if ((out->distinct + L.cur.n) * 10 > (L.mask + 1) * 6) {   /* keep the set below 60% */
      out->set_full = 1;
      break;
    }
  }
  L.done = 1;
  pthread_barrier_wait(&L.start);
  for (int t = 0; t < threads; t++) pthread_join(T[t], NULL);
  out->complete = L.cur.n == 0;
  out->seconds = elapsed_since(&L.t0);
  out->threads = threads;
  pthread_barrier_destroy(&L.start);
  pthread_barrier_destroy(&L.end);
  for (int t = 0; t < threads; t++) free(W[t].out.v);
  free(W); free(T); free(L.cur.v);
  munmap(mem, bytes);
  return out->seconds > 0 ? out->distinct / out->seconds : 0;
}
