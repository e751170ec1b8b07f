// spec_abi.hip — host entry points over the lowered spec (kc_spec_*), the
// TLA+-style state printer used for counterexample traces, and the C-ABI
// error plumbing.  Host code only: this is how traces are replayed from
// parent pointers and how the parity tests reach the spec lowering without
// a GPU.  It is NOT a model-checking fallback: the BFS itself only runs in
// the HIP engine (engine.hip).
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../../include/kubecheck.h"
#include "engine.h"
#include "engine_util.h"
#include "kc_common.h"
#include "kubeapi_spec.h"
#include "record.h"

namespace kc {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
}
const char* last_error() { return g_err; }

namespace {

template <class F>
int with_model(int nc, int np, int ns, F&& f) {
#define KC_DISPATCH(a, b, c) \
  if (nc == a && np == b && ns == c) return f(Model<a, b, c>{});
  KC_FOR_EACH_MODEL(KC_DISPATCH)
#undef KC_DISPATCH
  set_error("unsupported model nc=%d np=%d ns=%d", nc, np, ns);
  return -EINVAL;
}

std::string proc_name(int p, int nc, int np, int ns) {
  const char* base;
  int idx, cnt;
  if (p < nc) { base = "Client"; idx = p; cnt = nc; }
  else if (p < nc + np) { base = "PVCController"; idx = p - nc; cnt = np; }
  else { base = "Server"; idx = p - nc - np; cnt = ns; }
  return cnt == 1 ? std::string(base) : std::string(base) + std::to_string(idx + 1);
}

const char* kLabel[L_COUNT] = {"?", "CStart", "C1", "C10", "C11", "c12", "C13", "C2", "C3",
                               "C8", "C6", "C7", "C4", "C5", "PVCStart", "PVCListedPVCs",
                               "PVCHavePVCs", "PVCDone", "APIStart", "DoRequest", "DoReply",
                               "DoListRequest", "DoListReply"};
const char* kVerb[6] = {"defaultInitValue", "\"Create\"", "\"Get\"", "\"Update\"", "\"Delete\"",
                        "\"Force\""};
const char* kResp[4] = {"?", "\"Pending\"", "\"Ok\"", "\"Error\""};
const char* kKind[3] = {"defaultInitValue", "\"Secret\"", "\"PVC\""};

struct Printer {
  int nc, np, ns, A;
  std::string s;
  std::string pn(int p) const { return proc_name(p, nc, np, ns); }
  void procs(uint64_t vv) {
    s += "{";
    bool first = true;
    for (int c = 0; c < A; ++c)
      if ((vv >> c) & 1) { s += first ? "" : ", "; s += "\"" + pn(c) + "\""; first = false; }
    s += "}";
  }
  // object value from the tuple's oval byte
  void obj(uint64_t ov) {
    if (!(ov & 1)) { s += "defaultInitValue"; return; }
    const bool secret = ((ov >> 1) & 1) == ID_Secret;
    s += std::string("[k |-> \"") + (secret ? "Secret" : "PVC") + "\", n |-> \"" +
         (secret ? "foo" : "mypvc") + "\"";
    if ((ov >> 3) & 1) s += std::string(", spec |-> [pvname |-> \"") + (secret ? "foo" : "mypvc") + "\"]";
    if ((ov >> 2) & 1) { s += ", vv |-> "; procs((ov >> 4) & 15); }
    s += "]";
  }
  void uset(uint64_t set) {
    s += "{";
    bool first = true;
    for (int u = 0; u < 64; ++u) {
      if (!((set >> u) & 1)) continue;
      const int id = (u >> (A + 1)) & 1, spec = (u >> A) & 1, vv = u & ((1 << A) - 1);
      if (!first) s += ", ";
      first = false;
      obj(1u | (id << 1) | (1u << 2) | (spec << 3) | (vv << 4));
    }
    s += "}";
  }
};

}  // namespace

std::string format_tuple(const uint64_t* t, int nc, int np, int ns, bool ghost) {
  Printer pr{nc, np, ns, nc + np, {}};
  const int P = nc + np + ns;
  auto q = [&](int p, int k) { return t[1 + 19 * p + k]; };
  std::string& s = pr.s;
  s += "/\\ apiState = ";
  pr.uset(t[0] & ~GHOST_LOST);
  s += "\n/\\ requests = ";
  bool first = true;
  for (int p = 0; p < P; ++p) {
    if (!q(p, 11)) continue;
    s += first ? "(" : " @@ ";
    first = false;
    s += "\"" + pr.pn(p) + "\" :> [op |-> " + kVerb[q(p, 12) % 6] + ", obj |-> ";
    pr.obj(q(p, 14));
    s += std::string(", status |-> ") + kResp[q(p, 13) & 3] + "]";
  }
  s += first ? "<<>>" : ")";
  s += "\n/\\ listRequests = ";
  first = true;
  for (int p = 0; p < P; ++p) {
    if (!q(p, 15)) continue;
    s += first ? "(" : " @@ ";
    first = false;
    s += "\"" + pr.pn(p) + "\" :> [kind |-> " + kKind[q(p, 16) % 3] + ", objs |-> ";
    pr.uset(q(p, 18));
    s += std::string(", status |-> ") + kResp[q(p, 17) & 3] + "]";
  }
  s += first ? "<<>>" : ")";
  auto per_proc = [&](const char* var, auto&& val) {
    s += std::string("\n/\\ ") + var + " = (";
    for (int p = 0; p < P; ++p) {
      if (p) s += " @@ ";
      s += "\"" + pr.pn(p) + "\" :> ";
      val(p);
    }
    s += ")";
  };
  per_proc("pc", [&](int p) { s += std::string("\"") + kLabel[q(p, 0) % L_COUNT] + "\""; });
  per_proc("stack", [&](int p) {
    if (!q(p, 5)) { s += "<<>>"; return; }
    if (q(p, 6) == PR_API) {
      s += std::string("<<[procedure |-> \"API\", pc |-> \"") + kLabel[q(p, 7) % L_COUNT] +
           "\", op |-> " + kVerb[q(p, 8) % 6] + ", obj |-> ";
      pr.obj(q(p, 9));
      s += "]>>";
    } else {
      s += std::string("<<[procedure |-> \"ListAPI\", pc |-> \"") + kLabel[q(p, 7) % L_COUNT] +
           "\", kind |-> " + kKind[q(p, 10) % 3] + "]>>";
    }
  });
  per_proc("op", [&](int p) { s += kVerb[q(p, 1) % 6]; });
  per_proc("obj", [&](int p) { pr.obj(q(p, 2)); });
  per_proc("kind", [&](int p) { s += kKind[q(p, 3) % 3]; });
  s += "\n/\\ shouldReconcile = (";
  for (int p = 0; p < nc; ++p) {
    if (p) s += " @@ ";
    s += "\"" + pr.pn(p) + "\" :> " + (q(p, 4) ? "TRUE" : "FALSE");
  }
  s += ")\n";
  // the history variable of the build-defined NoLostUpdate (kubeapi_spec.h)
  if (ghost) s += std::string("/\\ lostUpdate = ") + ((t[0] & GHOST_LOST) ? "TRUE" : "FALSE") + "\n";
  return s;
}

}  // namespace kc

using namespace kc;

extern "C" {

const char* kc_last_error(void) { return kc::last_error(); }
int kc_abi_version(void) { return KC_ABI_VERSION; }
const char* kc_build_info(void) {
  return "kubecheck " __DATE__ " " __TIME__ " gfx950";
}
int kc_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int kc_spec_tuple_words(int nc, int np, int ns) {
  return with_model(nc, np, ns, [](auto m) { return decltype(m)::TUPLE_WORDS; });
}
int kc_spec_state_words(int nc, int np, int ns) {
  return with_model(nc, np, ns, [](auto m) { return decltype(m)::W; });
}

int kc_spec_init(const kc_model_config* cfg, uint64_t* out, int cap) {
  if (!cfg) { set_error("kc_spec_init: NULL"); return -EINVAL; }
  return with_model(cfg->nc, cfg->np, cfg->ns, [&](auto m) {
    using M = decltype(m);
    const int n = M::num_init();
    for (int k = 0; k < n && k < cap; ++k) {
      typename M::State s;
      M::init_state(k, s, cfg->variant);
      if (out) M::to_tuple(s, out + (size_t)k * M::TUPLE_WORDS);
    }
    return n;
  });
}

int kc_spec_successors(const kc_model_config* cfg, const uint64_t* tuple, int* actions,
                       uint64_t* succ, int cap, int* fail_action) {
  if (!cfg || !tuple) { set_error("kc_spec_successors: NULL"); return -EINVAL; }
  return with_model(cfg->nc, cfg->np, cfg->ns, [&](auto m) {
    using M = decltype(m);
    typename M::State s;
    if (!M::from_tuple(tuple, s)) { set_error("kc_spec_successors: tuple outside the lowered domain"); return -EINVAL; }
    const Flags f = flags_of(*cfg);
    const typename M::Plan pl = M::plan(s, f);
    if (fail_action) *fail_action = pl.fail_pos >= 0 ? M::slot_action(s, pl.fail_slot) : -1;
    for (int t = 0; t < pl.total && t < cap; ++t) {
      int slot, j;
      M::locate(pl, t, slot, j);
      typename M::State x;
      M::apply(s, slot, j, f, x);
      if (actions) actions[t] = M::slot_action(s, slot);
      if (succ) M::to_tuple(x, succ + (size_t)t * M::TUPLE_WORDS);
    }
    return pl.fail_pos >= 0 ? -2 : pl.total;
  });
}

int kc_spec_check(const kc_model_config* cfg, const uint64_t* tuple) {
  if (!cfg || !tuple) { set_error("kc_spec_check: NULL"); return -EINVAL; }
  return with_model(cfg->nc, cfg->np, cfg->ns, [&](auto m) {
    using M = decltype(m);
    typename M::State s;
    if (!M::from_tuple(tuple, s)) { set_error("kc_spec_check: bad tuple"); return -EINVAL; }
    return M::check(s, flags_of(*cfg).inv_mask);
  });
}

int kc_spec_fingerprint(const kc_model_config* cfg, const uint64_t* tuple, uint64_t* fp) {
  if (!cfg || !tuple || !fp) { set_error("kc_spec_fingerprint: NULL"); return -EINVAL; }
  return with_model(cfg->nc, cfg->np, cfg->ns, [&](auto m) {
    using M = decltype(m);
    typename M::State s;
    if (!M::from_tuple(tuple, s)) { set_error("kc_spec_fingerprint: bad tuple"); return -EINVAL; }
    *fp = M::fingerprint(s);
    return 0;
  });
}

int kc_spec_fp_selfcheck(const kc_model_config* cfg, const uint64_t* tuple) {
  if (!cfg || !tuple) { set_error("kc_spec_fp_selfcheck: NULL"); return -EINVAL; }
  return with_model(cfg->nc, cfg->np, cfg->ns, [&](auto m) {
    using M = decltype(m);
    typename M::State s;
    if (!M::from_tuple(tuple, s)) { set_error("kc_spec_fp_selfcheck: bad tuple"); return -EINVAL; }
    const Flags f = flags_of(*cfg);
    const typename M::Plan pl = M::plan(s, f);
    const uint64_t fold = M::fp_fold(s);
    int bad = 0;
    // the loop-free slot lookup (KC_LOCATE_SWAR) agrees with locate(), the
    // top byte (the dealt parent's index in k_claim) left alone
    const uint64_t cum = M::CUM_OK ? M::plan_cum(pl.counts | (0xa5ull << 56)) : 0;
    if (M::CUM_OK && (cum >> 56) != 0xa5) ++bad;
    for (int t = 0; t < pl.total; ++t) {
      int slot, j, who;
      M::locate(pl, t, slot, j);
      if (M::CUM_OK) {
        int s2, j2;
        M::locate_cum(cum, t, s2, j2);
        bad += (s2 != slot) + (j2 != j);
      }
      typename M::State x;
      M::apply(s, slot, j, f, x, who);
      if (M::fingerprint_succ(s, fold, x, who) != M::fingerprint(x)) ++bad;
      // the sharded path's owner projection (incremental from the parent's)
      const uint64_t fp1 = M::template fingerprint<1>(x);
      if (M::template fingerprint_succ<1>(s, fold, x, who, M::owner_proj(s)) != fp1) ++bad;
      // the record staging's owner at R = 2^k (owner_bits_succ >> (4 - k))
      // is the fingerprint's owner floor(fp * R / 2^63)
      const uint32_t ob = M::owner_bits_succ(s, x, who, M::owner_proj(s));
      for (int k = 0; k <= 3; ++k) {
        const uint64_t R = 1ull << k;
        if ((uint64_t)(ob >> (4 - k)) != (uint64_t)(((unsigned __int128)(fp1 << 1) * R) >> 64)) ++bad;
      }
      // the sharded path's exchange record round-trips the successor exactly
      uint64_t r[Record<M>::RW];
      const uint64_t key = 0x9e3779b97f4a7c15ull * (uint64_t)(t + 1);
      record_pack<M>(x, key, r);
      typename M::State y;
      uint64_t k2;
      record_unpack<M>(r, y, k2);
      for (int i = 0; i < M::W; ++i) bad += y.w[i] != x.w[i];
      bad += k2 != key;
    }
    return bad;
  });
}

int kc_spec_pack(const kc_model_config* cfg, const uint64_t* tuple, uint64_t* packed) {
  if (!cfg || !tuple || !packed) { set_error("kc_spec_pack: NULL"); return -EINVAL; }
  return with_model(cfg->nc, cfg->np, cfg->ns, [&](auto m) {
    using M = decltype(m);
    typename M::State s;
    if (!M::from_tuple(tuple, s)) { set_error("kc_spec_pack: bad tuple"); return -EINVAL; }
    for (int i = 0; i < M::W; ++i) packed[i] = s.w[i];
    return M::W;
  });
}

int kc_spec_unpack(const kc_model_config* cfg, const uint64_t* packed, uint64_t* tuple) {
  if (!cfg || !packed || !tuple) { set_error("kc_spec_unpack: NULL"); return -EINVAL; }
  return with_model(cfg->nc, cfg->np, cfg->ns, [&](auto m) {
    using M = decltype(m);
    typename M::State s;
    for (int i = 0; i < M::W; ++i) s.w[i] = packed[i];
    M::to_tuple(s, tuple);
    return M::TUPLE_WORDS;
  });
}

}  // extern "C"
