// ============================================================================
// ORACLE — CPU restatement of kube-batch's allocate hot path.
//
// TEST INFRASTRUCTURE ONLY. Nothing in the product (scheduler_amd/, libkbgpu)
// links, loads or calls this file; only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg do, and only as the checker / CPU baseline.
//
// Reference: /root/reference (kube-batch v0.4.2 / Volcano fork) with its
// vendored k8s.io/kubernetes v1.13.2. Every function cites the file:line it
// restates. The reference is Go and no Go toolchain exists in this image, so the
// reference itself cannot be run here; parity is pinned by
// the reference's own unit tests restated as known-answer tests
// (tests/test_oracle_kat.py) plus hand-derived vectors from the vendored formulas.
//
// Determinism decisions, applied identically to the GPU
// path: node order = nodes sorted by name (the reference iterates a Go map,
// util/scheduler_helper.go:161-167); SelectBestNode tie-break = lowest node
// index instead of rand.Intn (scheduler_helper.go:147-158); jobs are pushed in
// UID order (allocate.go:48 iterates a map); proportion iterates queues in UID
// order (proportion.go:101-154 iterates a map).
// ============================================================================
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "json.h"

namespace oracle {

using Labels = std::map<std::string, std::string>;
using oj::Value;

struct Panic : std::runtime_error {
  explicit Panic(const std::string& m) : std::runtime_error(m) {}
};

// ---------------------------------------------------------------------------
// k8s validation helpers (vendor/k8s.io/apimachinery/pkg/util/validation/validation.go:42-144)
// ---------------------------------------------------------------------------
static bool is_alnum(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9'); }
// qualifiedNameFmt = ([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9]  (validation.go:30-32)
static bool match_qualified_name_fmt(const std::string& s) {
  if (s.empty()) return false;
  if (!is_alnum(s.front()) || !is_alnum(s.back())) return false;
  for (char c : s)
    if (!(is_alnum(c) || c == '-' || c == '_' || c == '.')) return false;
  return true;
}
// dns1123SubdomainFmt (validation.go:108-131), the regex alone (the length rule is separate)
static bool match_dns1123_subdomain(const std::string& s) {
  if (s.empty()) return false;
  size_t start = 0;
  while (true) {
    size_t dot = s.find('.', start);
    std::string lab = s.substr(start, dot == std::string::npos ? std::string::npos : dot - start);
    if (lab.empty()) return false;
    auto lower_alnum = [](char c) { return (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9'); };
    if (!lower_alnum(lab.front()) || !lower_alnum(lab.back())) return false;
    for (char c : lab)
      if (!(lower_alnum(c) || c == '-')) return false;
    if (dot == std::string::npos) break;
    start = dot + 1;
  }
  return true;
}
// RegexError (validation.go:347-362), double spaces included
static std::string regex_error(const std::string& msg, const std::string& fmt, std::vector<std::string> ex) {
  if (ex.empty()) return msg + " (regex used for validation is '" + fmt + "')";
  std::string m = msg + " (e.g. ";
  for (size_t i = 0; i < ex.size(); ++i) m += (i ? " or " : "") + std::string("'") + ex[i] + "', ";
  return m + "regex used for validation is '" + fmt + "')";
}
static const char* kQNameFmt = "([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9]";
static const char* kQNameMsg =
    "must consist of alphanumeric characters, '-', '_' or '.', and must start and end with an alphanumeric character";
// IsQualifiedName (validation.go:42-71): the error list
static std::vector<std::string> qualified_name_errs(const std::string& v) {
  std::vector<std::string> parts, errs;
  size_t st = 0;
  while (true) {
    size_t sl = v.find('/', st);
    parts.push_back(v.substr(st, sl == std::string::npos ? std::string::npos : sl - st));
    if (sl == std::string::npos) break;
    st = sl + 1;
  }
  std::string name;
  if (parts.size() == 1) {
    name = parts[0];
  } else if (parts.size() == 2) {
    name = parts[1];
    if (parts[0].empty()) {
      errs.push_back("prefix part must be non-empty");
    } else {  // IsDNS1123Subdomain (:135-144), messages prefixed
      if (parts[0].size() > 253) errs.push_back("prefix part must be no more than 253 characters");
      if (!match_dns1123_subdomain(parts[0]))
        errs.push_back("prefix part " + regex_error("a DNS-1123 subdomain must consist of lower case alphanumeric "
                                                    "characters, '-' or '.', and must start and end with an "
                                                    "alphanumeric character",
                                                    "[a-z0-9]([-a-z0-9]*[a-z0-9])?(\\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*",
                                                    {"example.com"}));
    }
  } else {
    errs.push_back("a qualified name " + regex_error(kQNameMsg, kQNameFmt, {"MyName", "my.name", "123-abc"}) +
                   " with an optional DNS subdomain prefix and '/' (e.g. 'example.com/MyName')");
    return errs;
  }
  if (name.empty()) errs.push_back("name part must be non-empty");
  else if (name.size() > 63) errs.push_back("name part must be no more than 63 characters");
  if (!match_qualified_name_fmt(name))
    errs.push_back("name part " + regex_error(kQNameMsg, kQNameFmt, {"MyName", "my.name", "123-abc"}));
  return errs;
}
static bool is_qualified_name(const std::string& v) { return qualified_name_errs(v).empty(); }
// IsValidLabelValue (validation.go:97-106)
static std::vector<std::string> label_value_errs(const std::string& v) {
  std::vector<std::string> errs;
  if (v.size() > 63) errs.push_back("must be no more than 63 characters");
  if (!(v.empty() || match_qualified_name_fmt(v)))
    errs.push_back(regex_error("a valid label must be an empty string or consist of alphanumeric characters, '-', "
                               "'_' or '.', and must start and end with an alphanumeric character",
                               std::string("(") + kQNameFmt + ")?", {"MyValue", "my_value", "12345"}));
  return errs;
}
static bool is_valid_label_value(const std::string& v) { return label_value_errs(v).empty(); }
static std::string join(const std::vector<std::string>& v, const char* sep) {
  std::string o;
  for (size_t i = 0; i < v.size(); ++i) o += (i ? sep : "") + v[i];
  return o;
}
// fmt %q of a printable ASCII string (strconv.Quote)
static std::string go_quote(const std::string& s) {
  std::string o = "\"";
  for (char c : s) {
    if (c == '"' || c == '\\') o += '\\';
    o += c;
  }
  return o + "\"";
}

// IsScalarResourceName and friends (vendor/k8s.io/kubernetes/pkg/apis/core/v1/helper/helpers.go:36-104)
static bool contains(const std::string& s, const std::string& sub) { return s.find(sub) != std::string::npos; }
static bool has_prefix(const std::string& s, const std::string& p) { return s.compare(0, p.size(), p) == 0; }
static bool is_prefixed_native(const std::string& n) { return contains(n, "kubernetes.io/"); }
static bool is_native(const std::string& n) { return !contains(n, "/") || is_prefixed_native(n); }
static bool is_extended(const std::string& n) {
  if (is_native(n) || has_prefix(n, "requests.")) return false;
  return is_qualified_name("requests." + n);
}
static bool is_scalar_resource_name(const std::string& n) {
  return is_extended(n) || has_prefix(n, "hugepages-") || is_prefixed_native(n) || has_prefix(n, "attachable-volumes-");
}

// ---------------------------------------------------------------------------
// api.Resource (pkg/scheduler/api/resource_info.go:30-360)
// ---------------------------------------------------------------------------
static const double kMinMilliCPU = 10;                 // resource_info.go:70
static const double kMinMilliScalar = 10;              // resource_info.go:71
static const double kMinMemory = 10 * 1024 * 1024;     // resource_info.go:72

struct Resource {
  double cpu = 0, mem = 0;
  bool has_map = false;  // ScalarResources != nil
  std::map<std::string, double> sc;
  int max_task = 0;

  // NewResource (resource_info.go:75-93); quantities arrive pre-converted
  // (cpu/scalars in milli-units, memory/pods in units).
  static Resource from_list(const Value& rl) {
    Resource r;
    if (rl.kind != Value::Obj) return r;
    for (auto& kv : rl.o) {
      const std::string& n = kv.first;
      int64_t q = kv.second.as_int();
      if (n == "cpu") r.cpu += (double)q;
      else if (n == "memory") r.mem += (double)q;
      else if (n == "pods") r.max_task += (int)q;
      else if (is_scalar_resource_name(n)) r.add_scalar(n, (double)q);
    }
    return r;
  }
  void add_scalar(const std::string& n, double q) { set_scalar(n, get_sc(n) + q); }  // :351-353
  void set_scalar(const std::string& n, double q) { has_map = true; sc[n] = q; }     // :355-360
  double get_sc(const std::string& n) const {
    auto it = sc.find(n);
    return it == sc.end() ? 0.0 : it->second;
  }
  // IsEmpty (:96-108)
  bool is_empty() const {
    if (!(cpu < kMinMilliCPU && mem < kMinMemory)) return false;
    for (auto& kv : sc)
      if (kv.second >= kMinMilliScalar) return false;
    return true;
  }
  // IsZero (:111-128)
  bool is_zero(const std::string& rn) const {
    if (rn == "cpu") return cpu < kMinMilliCPU;
    if (rn == "memory") return mem < kMinMemory;
    if (!has_map) return true;
    if (!sc.count(rn)) throw Panic("unknown resource " + rn);
    return sc.at(rn) < kMinMilliScalar;
  }
  // Add (:131-143)
  Resource& add(const Resource& rr) {
    cpu += rr.cpu;
    mem += rr.mem;
    for (auto& kv : rr.sc) {
      has_map = true;
      sc[kv.first] += kv.second;
    }
    return *this;
  }
  // Sub (:145-159) -- assert.Assertf panics by default (util/assert/assert.go:17-40)
  Resource& sub(const Resource& rr) {
    if (!rr.less_equal(*this)) throw Panic("resource is not sufficient to do operation");
    cpu -= rr.cpu;
    mem -= rr.mem;
    for (auto& kv : rr.sc) {
      if (!has_map) return *this;
      sc[kv.first] -= kv.second;
    }
    return *this;
  }
  // SetMaxResource (:162-190)
  void set_max(const Resource& rr) {
    if (rr.cpu > cpu) cpu = rr.cpu;
    if (rr.mem > mem) mem = rr.mem;
    for (auto& kv : rr.sc) {
      if (!has_map) {
        has_map = true;
        sc = rr.sc;
        return;
      }
      if (kv.second > get_sc(kv.first)) sc[kv.first] = kv.second;
    }
  }
  // FitDelta (:193-215)
  Resource& fit_delta(const Resource& rr) {
    if (rr.cpu > 0) cpu -= rr.cpu + kMinMilliCPU;
    if (rr.mem > 0) mem -= rr.mem + kMinMemory;
    for (auto& kv : rr.sc) {
      has_map = true;
      if (kv.second > 0) sc[kv.first] -= kv.second + kMinMilliScalar;
    }
    return *this;
  }
  // Multi (:218-225)
  Resource& multi(double ratio) {
    cpu = cpu * ratio;
    mem = mem * ratio;
    for (auto& kv : sc) kv.second = kv.second * ratio;
    return *this;
  }
  // Less (:228-251)
  bool less(const Resource& rr) const {
    if (!(cpu < rr.cpu && mem < rr.mem)) return false;
    if (!has_map) return rr.has_map;
    for (auto& kv : sc) {
      if (!rr.has_map) return false;
      if (kv.second >= rr.get_sc(kv.first)) return false;
    }
    return true;
  }
  // LessEqual (:253-276)
  bool less_equal(const Resource& rr) const {
    bool is_less = (cpu < rr.cpu || std::fabs(rr.cpu - cpu) < kMinMilliCPU) &&
                   (mem < rr.mem || std::fabs(rr.mem - mem) < kMinMemory);
    if (!is_less) return false;
    if (!has_map) return true;
    for (auto& kv : sc) {
      if (!rr.has_map) return false;
      double rq = rr.get_sc(kv.first);
      if (!(kv.second < rq || std::fabs(rq - kv.second) < kMinMilliScalar)) return false;
    }
    return true;
  }
  // Get (:316-330)
  double get(const std::string& rn) const {
    if (rn == "cpu") return cpu;
    if (rn == "memory") return mem;
    if (!has_map) return 0;
    return get_sc(rn);
  }
  // ResourceNames (:333-341)
  std::vector<std::string> names() const {
    std::vector<std::string> v = {"cpu", "memory"};
    for (auto& kv : sc) v.push_back(kv.first);
    return v;
  }
  Value to_json() const {
    Value v;
    v.kind = Value::Obj;
    Value c; c.kind = Value::Dbl; c.d = cpu;
    Value m; m.kind = Value::Dbl; m.d = mem;
    v.o.emplace_back("cpu", c);
    v.o.emplace_back("memory", m);
    if (has_map) {
      Value s; s.kind = Value::Obj;
      for (auto& kv : sc) { Value x; x.kind = Value::Dbl; x.d = kv.second; s.o.emplace_back(kv.first, x); }
      v.o.emplace_back("scalars", s);
    } else {
      v.o.emplace_back("scalars", Value());
    }
    Value mt; mt.kind = Value::Int; mt.i = max_task;
    v.o.emplace_back("maxTaskNum", mt);
    return v;
  }
  static Resource from_json(const Value& v) {  // inverse of to_json, for KATs
    Resource r;
    r.cpu = v.get("cpu") ? v.get("cpu")->as_dbl() : 0;
    r.mem = v.get("memory") ? v.get("memory")->as_dbl() : 0;
    r.max_task = (int)v.int_at("maxTaskNum");
    const Value* s = v.get("scalars");
    if (s && s->kind == Value::Obj) {
      r.has_map = true;
      for (auto& kv : s->o) r.sc[kv.first] = kv.second.as_dbl();
    }
    return r;
  }
};

// helpers.Min / helpers.Share (pkg/scheduler/api/helpers/helpers.go:27-63)
static Resource res_min(const Resource& l, const Resource& r) {
  Resource res;
  res.cpu = std::min(l.cpu, r.cpu);
  res.mem = std::min(l.mem, r.mem);
  if (!l.has_map || !r.has_map) return res;
  res.has_map = true;
  for (auto& kv : l.sc) res.sc[kv.first] = std::min(kv.second, r.get_sc(kv.first));
  return res;
}
static double share(double l, double r) {
  if (r == 0) return l == 0 ? 0 : 1;
  return l / r;
}

// ---------------------------------------------------------------------------
// labels.Selector (vendor/k8s.io/apimachinery/pkg/labels/selector.go)
// ---------------------------------------------------------------------------
enum Op { OP_IN, OP_NOTIN, OP_EXISTS, OP_DNE, OP_GT, OP_LT, OP_EQ, OP_NEQ };

struct Requirement {
  std::string key;
  Op op;
  std::vector<std::string> vals;
  bool has_value(const std::string& v) const {
    for (auto& x : vals)
      if (x == v) return true;
    return false;
  }
  // Requirement.Matches (selector.go:185-236)
  bool matches(const Labels& ls) const {
    auto it = ls.find(key);
    bool has = it != ls.end();
    switch (op) {
      case OP_IN: case OP_EQ: return has && has_value(it->second);
      case OP_NOTIN: case OP_NEQ: return !has || !has_value(it->second);
      case OP_EXISTS: return has;
      case OP_DNE: return !has;
      case OP_GT: case OP_LT: {
        if (!has) return false;
        int64_t lv, rv;
        if (!parse_int64(it->second, &lv)) return false;
        if (vals.size() != 1) return false;
        if (!parse_int64(vals[0], &rv)) return false;
        return (op == OP_GT && lv > rv) || (op == OP_LT && lv < rv);
      }
    }
    return false;
  }
  // strconv.ParseInt(s, 10, 64)
  static bool parse_int64(const std::string& s, int64_t* out) {
    if (s.empty()) return false;
    size_t i = 0;
    bool neg = false;
    if (s[0] == '+' || s[0] == '-') { neg = s[0] == '-'; i = 1; }
    if (i >= s.size()) return false;
    unsigned long long acc = 0;
    const unsigned long long lim = neg ? 9223372036854775808ULL : 9223372036854775807ULL;
    for (; i < s.size(); ++i) {
      if (s[i] < '0' || s[i] > '9') return false;
      unsigned d = s[i] - '0';
      if (acc > (lim - d) / 10) return false;
      acc = acc * 10 + d;
    }
    *out = neg ? (int64_t)(0 - acc) : (int64_t)acc;
    return true;
  }
};

// NewRequirement (selector.go:133-170); returns false on validation error (its text in *err).
static bool new_requirement(const std::string& key, Op op, const std::vector<std::string>& vals, Requirement* out,
                            std::string* err = nullptr) {
  auto bad = [&](const std::string& m) {
    if (err) *err = m;
    return false;
  };
  {  // validateLabelKey (:833-838)
    auto e = qualified_name_errs(key);
    if (!e.empty()) return bad("invalid label key " + go_quote(key) + ": " + join(e, "; "));
  }
  switch (op) {
    case OP_IN: case OP_NOTIN:
      if (vals.empty()) return bad("for 'in', 'notin' operators, values set can't be empty");
      break;
    case OP_EQ: case OP_NEQ:
      if (vals.size() != 1) return bad("exact-match compatibility requires one single value");
      break;
    case OP_EXISTS: case OP_DNE:
      if (!vals.empty()) return bad("values set must be empty for exists and does not exist");
      break;
    case OP_GT: case OP_LT: {
      if (vals.size() != 1) return bad("for 'Gt', 'Lt' operators, exactly one value is required");
      int64_t tmp;
      if (!Requirement::parse_int64(vals[0], &tmp)) return bad("for 'Gt', 'Lt' operators, the value must be an integer");
      break;
    }
  }
  for (auto& v : vals) {  // validateLabelValue (:840-845)
    auto e = label_value_errs(v);
    if (!e.empty()) return bad("invalid label value: " + go_quote(v) + ": " + join(e, "; "));
  }
  out->key = key;
  out->op = op;
  out->vals = vals;
  return true;
}

struct Selector {
  enum Kind { LIST, NOTHING } kind = LIST;  // an empty LIST is Everything()
  std::vector<Requirement> reqs;
  bool matches(const Labels& ls) const {
    if (kind == NOTHING) return false;
    for (auto& r : reqs)
      if (!r.matches(ls)) return false;
    return true;
  }
  static Selector nothing() { Selector s; s.kind = NOTHING; return s; }
  static Selector everything() { return Selector(); }
};

// SelectorFromSet (selector.go:849-866): any invalid pair => Everything().
static Selector selector_from_set(const Labels& set) {
  Selector s;
  for (auto& kv : set) {
    Requirement r;
    if (!new_requirement(kv.first, OP_EQ, {kv.second}, &r)) return Selector::everything();
    s.reqs.push_back(r);
  }
  return s;
}

struct SelReq {  // v1.NodeSelectorRequirement / metav1.LabelSelectorRequirement
  std::string key, op;
  std::vector<std::string> values;
};
static std::vector<SelReq> parse_reqs(const Value& arr) {
  std::vector<SelReq> out;
  if (arr.kind != Value::Arr) return out;
  for (auto& e : arr.a) {
    SelReq r;
    r.key = e.str_at("key");
    r.op = e.str_at("operator");
    for (auto& x : e.arr_at("values")) r.values.push_back(x.as_str());
    out.push_back(r);
  }
  return out;
}

// NodeSelectorRequirementsAsSelector (core/v1/helper/helpers.go:222-254)
static bool node_reqs_as_selector(const std::vector<SelReq>& nsm, Selector* out) {
  if (nsm.empty()) { *out = Selector::nothing(); return true; }
  Selector s;
  for (auto& e : nsm) {
    Op op;
    if (e.op == "In") op = OP_IN;
    else if (e.op == "NotIn") op = OP_NOTIN;
    else if (e.op == "Exists") op = OP_EXISTS;
    else if (e.op == "DoesNotExist") op = OP_DNE;
    else if (e.op == "Gt") op = OP_GT;
    else if (e.op == "Lt") op = OP_LT;
    else return false;
    Requirement r;
    if (!new_requirement(e.key, op, e.values, &r)) return false;
    s.reqs.push_back(r);
  }
  *out = s;
  return true;
}

// NodeSelectorRequirementsAsFieldSelector (helpers.go:258-285) evaluated against
// fields.Set{"metadata.name": node.Name} (algorithm/types.go:30-32).
static bool node_field_reqs_match(const std::vector<SelReq>& nsm, const std::string& node_name, bool* ok) {
  *ok = true;
  if (nsm.empty()) return false;  // fields.Nothing()
  bool all = true;
  for (auto& e : nsm) {
    if ((e.op != "In" && e.op != "NotIn") || e.values.size() != 1) { *ok = false; return false; }
    std::string fv = e.key == "metadata.name" ? node_name : std::string();
    bool m = e.op == "In" ? fv == e.values[0] : fv != e.values[0];
    all = all && m;
  }
  return all;
}

struct NodeSelTerm {
  std::vector<SelReq> exprs, fields;
};

// MatchNodeSelectorTerms (helpers.go:302-333)
static bool match_node_selector_terms(const std::vector<NodeSelTerm>& terms, const Labels& labels,
                                      const std::string& node_name) {
  for (auto& t : terms) {
    if (t.exprs.empty() && t.fields.empty()) continue;
    if (!t.exprs.empty()) {
      Selector s;
      if (!node_reqs_as_selector(t.exprs, &s) || !s.matches(labels)) continue;
    }
    if (!t.fields.empty()) {
      bool ok;
      bool m = node_field_reqs_match(t.fields, node_name, &ok);
      if (!ok || !m) continue;
    }
    return true;
  }
  return false;
}

struct LabelSelector {  // *metav1.LabelSelector
  bool present = false;
  Labels match_labels;
  std::vector<SelReq> exprs;
};

// LabelSelectorAsSelector (vendor/k8s.io/apimachinery/pkg/apis/meta/v1/helpers.go:31-67). matchLabels go in
// key order (a Go map: the order, and so which of several invalid pairs is reported, is random there).
static bool label_selector_as_selector(const LabelSelector& ps, Selector* out, std::string* err = nullptr) {
  if (!ps.present) { *out = Selector::nothing(); return true; }
  if (ps.match_labels.size() + ps.exprs.size() == 0) { *out = Selector::everything(); return true; }
  Selector s;
  for (auto& kv : ps.match_labels) {
    Requirement r;
    if (!new_requirement(kv.first, OP_EQ, {kv.second}, &r, err)) return false;
    s.reqs.push_back(r);
  }
  for (auto& e : ps.exprs) {
    Op op;
    if (e.op == "In") op = OP_IN;
    else if (e.op == "NotIn") op = OP_NOTIN;
    else if (e.op == "Exists") op = OP_EXISTS;
    else if (e.op == "DoesNotExist") op = OP_DNE;
    else {
      if (err) *err = go_quote(e.op) + " is not a valid pod selector operator";
      return false;
    }
    Requirement r;
    if (!new_requirement(e.key, op, e.values, &r, err)) return false;
    s.reqs.push_back(r);
  }
  *out = s;
  return true;
}

// ---------------------------------------------------------------------------
// v1 objects (restated fields only)
// ---------------------------------------------------------------------------
struct Port {
  int32_t host_port = 0;
  std::string host_ip, protocol;
};
struct Container {
  Value req;  // ResourceList (canonical integers), kept as JSON for key-presence tests
  std::vector<Port> ports;
};
struct Toleration {
  std::string key, op, value, effect;
};
struct Taint {
  std::string key, value, effect;
};
struct PodAffinityTerm {
  LabelSelector sel;
  std::vector<std::string> namespaces;
  std::string topology_key;
};
struct WeightedPodAffinityTerm {
  int32_t weight = 0;
  PodAffinityTerm term;
};
struct PodAffinity {  // used for both PodAffinity and PodAntiAffinity
  std::vector<PodAffinityTerm> required;
  std::vector<WeightedPodAffinityTerm> preferred;
};
struct NodeAffinity {
  bool has_required = false;
  std::vector<NodeSelTerm> required;
  std::vector<std::pair<int32_t, NodeSelTerm>> preferred;
};
struct Affinity {
  bool has_node = false, has_pod = false, has_anti = false;
  NodeAffinity node;
  PodAffinity pod, anti;
};

struct Pod {
  std::string ns, name, uid, node, phase, group;
  bool deleting = false;
  bool has_priority = false;
  int32_t priority = 0;
  int64_t ctime = 0;
  Labels labels;
  std::vector<Container> containers, init;
  Labels node_selector;
  std::vector<Toleration> tolerations;
  bool has_affinity = false;
  Affinity aff;
};

struct NodeSpec {
  std::string name;
  Labels labels;
  Value alloc, cap;
  std::vector<Taint> taints;
  bool unschedulable = false;
  std::vector<std::pair<std::string, std::string>> conditions;  // (type, status)
};

static Labels parse_labels(const Value* v) {
  Labels l;
  if (v && v->kind == Value::Obj)
    for (auto& kv : v->o) l[kv.first] = kv.second.as_str();
  return l;
}

static LabelSelector parse_label_selector(const Value* v) {
  LabelSelector s;
  if (!v || v->is_null()) return s;
  s.present = true;
  s.match_labels = parse_labels(v->get("matchLabels"));
  if (v->get("matchExpressions")) s.exprs = parse_reqs(*v->get("matchExpressions"));
  return s;
}

static PodAffinityTerm parse_pod_aff_term(const Value& v) {
  PodAffinityTerm t;
  t.sel = parse_label_selector(v.get("labelSelector"));
  for (auto& n : v.arr_at("namespaces")) t.namespaces.push_back(n.as_str());
  t.topology_key = v.str_at("topologyKey");
  return t;
}

static PodAffinity parse_pod_affinity(const Value& v) {
  PodAffinity pa;
  for (auto& t : v.arr_at("required")) pa.required.push_back(parse_pod_aff_term(t));
  for (auto& t : v.arr_at("preferred")) {
    WeightedPodAffinityTerm w;
    w.weight = (int32_t)t.int_at("weight");
    w.term = parse_pod_aff_term(*t.get("podAffinityTerm"));
    pa.preferred.push_back(w);
  }
  return pa;
}

static NodeSelTerm parse_node_sel_term(const Value& v) {
  NodeSelTerm t;
  if (v.get("matchExpressions")) t.exprs = parse_reqs(*v.get("matchExpressions"));
  if (v.get("matchFields")) t.fields = parse_reqs(*v.get("matchFields"));
  return t;
}

static Container parse_container(const Value& v) {
  Container c;
  if (v.get("req")) c.req = *v.get("req");
  for (auto& p : v.arr_at("ports")) {
    Port pt;
    pt.host_port = (int32_t)p.int_at("hostPort");
    pt.host_ip = p.str_at("hostIP");
    pt.protocol = p.str_at("protocol");
    c.ports.push_back(pt);
  }
  return c;
}

static Pod parse_pod(const Value& v) {
  Pod p;
  p.ns = v.str_at("ns");
  p.name = v.str_at("name");
  p.uid = v.str_at("uid");
  p.node = v.str_at("node");
  p.phase = v.str_at("phase");
  p.group = v.str_at("group");
  p.deleting = v.bool_at("deleting");
  if (v.has("priority")) { p.has_priority = true; p.priority = (int32_t)v.int_at("priority"); }
  p.ctime = v.int_at("ctime");
  p.labels = parse_labels(v.get("labels"));
  for (auto& c : v.arr_at("containers")) p.containers.push_back(parse_container(c));
  for (auto& c : v.arr_at("init")) p.init.push_back(parse_container(c));
  p.node_selector = parse_labels(v.get("nodeSelector"));
  for (auto& t : v.arr_at("tolerations")) {
    Toleration tol;
    tol.key = t.str_at("key");
    tol.op = t.str_at("operator");
    tol.value = t.str_at("value");
    tol.effect = t.str_at("effect");
    p.tolerations.push_back(tol);
  }
  const Value* a = v.get("affinity");
  if (a && !a->is_null()) {
    p.has_affinity = true;
    const Value* na = a->get("nodeAffinity");
    if (na && !na->is_null()) {
      p.aff.has_node = true;
      const Value* req = na->get("required");
      if (req && !req->is_null()) {
        p.aff.node.has_required = true;
        for (auto& t : req->a) p.aff.node.required.push_back(parse_node_sel_term(t));
      }
      for (auto& t : na->arr_at("preferred")) {
        const Value* pref = t.get("preference");
        p.aff.node.preferred.emplace_back((int32_t)t.int_at("weight"),
                                          pref ? parse_node_sel_term(*pref) : NodeSelTerm());
      }
    }
    const Value* pa = a->get("podAffinity");
    if (pa && !pa->is_null()) { p.aff.has_pod = true; p.aff.pod = parse_pod_affinity(*pa); }
    const Value* paa = a->get("podAntiAffinity");
    if (paa && !paa->is_null()) { p.aff.has_anti = true; p.aff.anti = parse_pod_affinity(*paa); }
  }
  return p;
}

static NodeSpec parse_node(const Value& v) {
  NodeSpec n;
  n.name = v.str_at("name");
  n.labels = parse_labels(v.get("labels"));
  if (v.get("alloc")) n.alloc = *v.get("alloc");
  if (v.get("cap")) n.cap = *v.get("cap");
  for (auto& t : v.arr_at("taints")) n.taints.push_back({t.str_at("key"), t.str_at("value"), t.str_at("effect")});
  n.unschedulable = v.bool_at("unschedulable");
  for (auto& c : v.arr_at("conditions")) n.conditions.emplace_back(c.str_at("type"), c.str_at("status"));
  return n;
}

// ---------------------------------------------------------------------------
// Task / Job / Node infos (pkg/scheduler/api)
// ---------------------------------------------------------------------------
enum TaskStatus {  // api/types.go:23-61
  Pending = 1 << 0, Allocated = 1 << 1, Pipelined = 1 << 2, Binding = 1 << 3, Bound = 1 << 4,
  Running = 1 << 5, Releasing = 1 << 6, Succeeded = 1 << 7, Failed = 1 << 8, Unknown = 1 << 9
};
static const char* status_name(int s) {
  switch (s) {
    case Pending: return "Pending"; case Allocated: return "Allocated"; case Pipelined: return "Pipelined";
    case Binding: return "Binding"; case Bound: return "Bound"; case Running: return "Running";
    case Releasing: return "Releasing"; case Succeeded: return "Succeeded"; case Failed: return "Failed";
  }
  return "Unknown";
}
// AllocatedStatus (api/helpers.go:72-79)
static bool allocated_status(int s) { return s == Bound || s == Binding || s == Running || s == Allocated; }
// getTaskStatus (api/helpers.go:35-69)
static int get_task_status(const Pod& p) {
  if (p.phase == "Running") return p.deleting ? Releasing : Running;
  if (p.phase == "Pending") {
    if (p.deleting) return Releasing;
    return p.node.empty() ? Pending : Bound;
  }
  if (p.phase == "Unknown") return Unknown;
  if (p.phase == "Succeeded") return Succeeded;
  if (p.phase == "Failed") return Failed;
  return Unknown;
}

// GetPodResourceWithoutInitContainers / GetPodResourceRequest (api/pod_info.go:53-73)
static Resource pod_resreq(const Pod& p) {
  Resource r;
  for (auto& c : p.containers) r.add(Resource::from_list(c.req));
  return r;
}
static Resource pod_initreq(const Pod& p) {
  Resource r = pod_resreq(p);
  for (auto& c : p.init) r.set_max(Resource::from_list(c.req));
  return r;
}

struct Task {  // api.TaskInfo (job_info.go:36-54, NewTaskInfo :69-95)
  std::string uid, job, name, ns, node_name;
  Resource resreq, initreq;
  int status = Pending;
  int32_t priority = 1;
  const Pod* pod = nullptr;
};

struct FitErrs {  // api.FitErrors (unschedule_info.go:22-79): only the histogram is observable
  std::map<std::string, int> hist;
};

struct Job {  // api.JobInfo (job_info.go:127-157)
  std::string uid, name, ns, queue, pg_phase;
  int32_t priority = 0, min_avail = 0;
  int64_t ctime = 0;
  bool has_pg = false;
  std::map<int, std::map<std::string, Task*>> tsi;  // TaskStatusIndex
  std::map<std::string, Task*> tasks;
  Resource allocated, total_request;
  std::map<std::string, FitErrs> fit_errors;  // NodesFitErrors

  void add_task_info(Task* t) {  // :239-248
    tasks[t->uid] = t;
    tsi[t->status][t->uid] = t;
    total_request.add(t->resreq);
    if (allocated_status(t->status)) allocated.add(t->resreq);
  }
  void delete_task_info(Task* t) {  // :265-283
    auto it = tasks.find(t->uid);
    if (it == tasks.end()) return;
    Task* task = it->second;
    total_request.sub(task->resreq);
    if (allocated_status(task->status)) allocated.sub(task->resreq);
    tasks.erase(it);
    auto s = tsi.find(task->status);
    if (s != tsi.end()) {
      s->second.erase(task->uid);
      if (s->second.empty()) tsi.erase(s);
    }
  }
  void update_task_status(Task* t, int status) {  // :251-263
    delete_task_info(t);
    t->status = status;
    add_task_info(t);
  }
  int32_t ready_task_num() const {  // :367-378
    int n = 0;
    for (auto& kv : tsi)
      if (allocated_status(kv.first) || kv.first == Succeeded) n += (int)kv.second.size();
    return n;
  }
  int32_t waiting_task_num() const {  // :381-390
    auto it = tsi.find(Pipelined);
    return it == tsi.end() ? 0 : (int32_t)it->second.size();
  }
  int32_t valid_task_num() const {  // :393-405
    int n = 0;
    for (auto& kv : tsi)
      if (allocated_status(kv.first) || kv.first == Succeeded || kv.first == Pipelined || kv.first == Pending)
        n += (int)kv.second.size();
    return n;
  }
  bool ready() const { return ready_task_num() >= min_avail; }                          // :408-412
  bool pipelined() const { return waiting_task_num() + ready_task_num() >= min_avail; }  // :415-419
};

struct QueueI {  // api.QueueInfo (queue_info.go)
  std::string uid, name;
  int32_t weight = 1;
  int64_t ctime = 0;
};

struct NodeI {  // api.NodeInfo (node_info.go:28-50)
  std::string name;
  const NodeSpec* node = nullptr;
  Resource releasing, idle, used, alloc, cap;
  std::set<std::string> task_keys;
  std::vector<const Task*> tasks;  // clones' sources (Pods() order is irrelevant)

  // AddTask (node_info.go:165-193)
  void add_task(const Task* t) {
    std::string key = t->pod->ns + "/" + t->pod->name;
    if (task_keys.count(key)) throw std::runtime_error("task already on node");
    switch (t->status) {
      case Releasing: releasing.add(t->resreq); idle.sub(t->resreq); break;
      case Pipelined: releasing.sub(t->resreq); break;
      default: idle.sub(t->resreq);
    }
    used.add(t->resreq);
    task_keys.insert(key);
    tasks.push_back(t);
  }
};

// ---------------------------------------------------------------------------
// schedulercache.NodeInfo (vendor/k8s.io/kubernetes/pkg/scheduler/cache/node_info.go)
// the predicates / nodeorder plugins' private per-node state.
// ---------------------------------------------------------------------------
struct PodRef {
  const Pod* pod;
  int node;  // index of the node named by pod.Spec.NodeName
};

// GetNonzeroRequests (vendor/.../priorities/util/non_zero.go:31-52)
static void nonzero_requests(const Value& req, int64_t* cpu, int64_t* mem) {
  const Value* c = req.get("cpu");
  const Value* m = req.get("memory");
  *cpu = c ? c->as_int() : 100;
  *mem = m ? m->as_int() : 200LL * 1024 * 1024;
}

struct HostPort {  // HostPortInfo key after sanitize (cache/host_ports.go:128-135)
  std::string ip, proto;
  int32_t port;
  bool operator<(const HostPort& o) const {
    return std::tie(ip, proto, port) < std::tie(o.ip, o.proto, o.port);
  }
};
static void sanitize(std::string* ip, std::string* proto) {
  if (ip->empty()) *ip = "0.0.0.0";
  if (proto->empty()) *proto = "TCP";
}

static bool has_pod_affinity_constraints(const Pod& p) {  // cache/node_info.go:492-495
  return p.has_affinity && (p.aff.has_pod || p.aff.has_anti);
}

struct KNode {
  const NodeSpec* node = nullptr;
  int idx = -1;
  std::vector<PodRef> pods, pods_with_affinity;
  int64_t nz_cpu = 0, nz_mem = 0;
  int64_t alloc_cpu = 0, alloc_mem = 0;
  std::multiset<HostPort> used_ports;
  std::string mem_pressure, disk_pressure, pid_pressure;

  // SetNode (cache/node_info.go:608-631)
  void set_node(const NodeSpec* n, int i) {
    node = n;
    idx = i;
    alloc_cpu = n->alloc.int_at("cpu");
    alloc_mem = n->alloc.int_at("memory");
    for (auto& c : n->conditions) {
      if (c.first == "MemoryPressure") mem_pressure = c.second;
      else if (c.first == "DiskPressure") disk_pressure = c.second;
      else if (c.first == "PIDPressure") pid_pressure = c.second;
    }
  }
  // AddPod (cache/node_info.go:498-520) + calculateResource (:578-591)
  void add_pod(const Pod* p, int node_of_pod) {
    for (auto& c : p->containers) {
      int64_t a, b;
      nonzero_requests(c.req, &a, &b);
      nz_cpu += a;
      nz_mem += b;
    }
    pods.push_back({p, node_of_pod});
    if (has_pod_affinity_constraints(*p)) pods_with_affinity.push_back({p, node_of_pod});
    // UpdateUsedPorts (:593-606) / HostPortInfo.Add (host_ports.go:50-66)
    for (auto& c : p->containers)
      for (auto& pt : c.ports) {
        if (pt.host_port <= 0) continue;
        HostPort hp{pt.host_ip, pt.protocol, pt.host_port};
        sanitize(&hp.ip, &hp.proto);
        if (!used_ports.count(hp)) used_ports.insert(hp);  // set semantics
      }
  }
  // HostPortInfo.CheckConflict (host_ports.go:96-125)
  bool check_conflict(std::string ip, std::string proto, int32_t port) const {
    if (port <= 0) return false;
    sanitize(&ip, &proto);
    if (ip == "0.0.0.0") {
      for (auto& u : used_ports)
        if (u.proto == proto && u.port == port) return true;
      return false;
    }
    return used_ports.count({"0.0.0.0", proto, port}) || used_ports.count({ip, proto, port});
  }
};

// ---------------------------------------------------------------------------
// Predicate failure reasons (vendor/.../algorithm/predicates/error.go:24-84, api/unschedule_info.go:11-19)
// ---------------------------------------------------------------------------
static const char* kResourceFit = "node(s) resource fit failed";
static const char* kPodNumberExceeded = "node(s) pod number exceeded";
static const char* kNodeNotReady = "node(s) were not ready";
static const char* kNodeOutOfDisk = "node(s) were out of disk space";
static const char* kNodeNetworkUnavailable = "node(s) had unavailable network";
static const char* kNodeUnschedulable = "node(s) were unschedulable";
static const char* kNodeSelectorNotMatch = "node(s) didn't match node selector";
static const char* kHostPorts = "node(s) didn't have free ports for the requested pod ports";
static const char* kTaints = "node(s) had taints that the pod didn't tolerate";
static const char* kMemPressure = "node(s) had memory pressure";
static const char* kDiskPressure = "node(s) had disk pressure";
static const char* kPIDPressure = "node(s) had pid pressure";
static const char* kPodAffinityNotMatch = "node(s) didn't match pod affinity/anti-affinity";
static const char* kPodAffinityRules = "node(s) didn't match pod affinity rules";
static const char* kPodAntiAffinityRules = "node(s) didn't match pod anti-affinity rules";
static const char* kExistingAntiAffinity = "node(s) didn't satisfy existing pods anti-affinity rules";

struct PredResult {
  bool ok = true;
  std::vector<std::string> reasons;  // FitError reasons, or [err.Error()] for a plain error
  static PredResult fail(std::vector<std::string> r) { PredResult p; p.ok = false; p.reasons = std::move(r); return p; }
};

// ---------------------------------------------------------------------------
// Session + plugins
// ---------------------------------------------------------------------------
struct PluginOpt {  // conf.PluginOption (conf/scheduler_conf.go:37-56)
  std::string name;
  bool job_order = false, job_ready = false, job_pipelined = false, task_order = false, preemptable = false,
       reclaimable = false, queue_order = false, predicate = false, node_order = false;
  std::map<std::string, std::string> args;
};

// Arguments.GetInt / GetBool (framework/arguments.go:26-66)
static void get_int(const std::map<std::string, std::string>& a, int* p, const std::string& k) {
  auto it = a.find(k);
  if (it == a.end() || it->second.empty()) return;
  int64_t v;
  if (!Requirement::parse_int64(it->second, &v)) return;
  *p = (int)v;
}
static void get_bool(const std::map<std::string, std::string>& a, bool* p, const std::string& k) {
  auto it = a.find(k);
  if (it == a.end() || it->second.empty()) return;
  const std::string& s = it->second;
  if (s == "1" || s == "t" || s == "T" || s == "TRUE" || s == "true" || s == "True") *p = true;
  else if (s == "0" || s == "f" || s == "F" || s == "FALSE" || s == "false" || s == "False") *p = false;
}

struct Event {
  std::string task_uid, node;
  int kind;  // Allocated or Pipelined
};

// workqueue.ParallelizeUntil(ctx, workers, pieces, fn) (client-go/util/workqueue/parallelizer.go:38-71):
// a persistent pool; each piece index is handed out once.
class Pool {
 public:
  explicit Pool(int workers) : workers_(std::max(1, workers)) {
    for (int i = 1; i < workers_; ++i) threads_.emplace_back([this] { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
      gen_++;
    }
    cv_.notify_all();
    for (auto& t : threads_) t.join();
  }
  void run(int n, const std::function<void(int)>& fn) {
    if (workers_ == 1 || n < 2) {
      for (int i = 0; i < n; ++i) fn(i);
      return;
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      fn_ = &fn;
      n_ = n;
      next_.store(0);
      active_ = (int)threads_.size();
      gen_++;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [this] { return active_ == 0; });
    fn_ = nullptr;
  }

 private:
  int workers_;
  std::vector<std::thread> threads_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* fn_ = nullptr;
  int n_ = 0;
  std::atomic<int> next_{0};
  int active_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
  void work() {  // pieces are handed out in grains of 32 indices
    for (;;) {
      int i = next_.fetch_add(32);
      if (i >= n_) break;
      int e = std::min(n_, i + 32);
      for (; i < e; ++i) (*fn_)(i);
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      work();
      {
        std::lock_guard<std::mutex> g(mu_);
        if (--active_ == 0) done_cv_.notify_all();
      }
    }
  }
};

struct Options {
  int workers = 1;          // ParallelizeUntil workers (reference: 16)
  bool literal_affinity = false;  // slow-path restatements of the inter-pod affinity code
  int64_t max_tasks = -1;   // bounded sample for the CPU baseline (-1 = all)
};

class Session {
 public:
  // ---- snapshot (cache/cache.go:584-654, event_handlers.go:42-100) ----
  std::vector<NodeSpec> node_specs;
  std::deque<Pod> pods;
  std::deque<Task> tasks;
  std::vector<NodeI> nodes;  // canonical: sorted by name
  std::map<std::string, int> node_index;
  std::map<std::string, Job> jobs;
  std::map<std::string, QueueI> queues;
  std::vector<std::vector<PluginOpt>> tiers;
  Options opt;

  // ---- plugin state ----
  std::set<std::string> plugins;
  bool has_lister = false;
  std::map<std::string, Task*> lister_tasks, lister_aff;  // plugins/util/util.go:34-82
  std::vector<KNode> knodes;                              // GenerateNodeMapAndSlice (util.go:186-198)
  bool mem_pressure = false, disk_pressure = false, pid_pressure = false;   // predicates.go:63-111
  int w_lr = 1, w_na = 1, w_pa = 1, w_bra = 1;                             // nodeorder.go:96-140
  Resource drf_total;
  std::map<std::string, Resource> drf_alloc;                              // drf.go:30-58
  std::map<std::string, double> drf_share;
  Resource prop_total;
  struct QAttr { std::string id, name; int32_t weight; double share = 0; Resource deserved, allocated, request; };
  std::map<std::string, QAttr> prop;                                      // proportion.go:33-44

  // ---- outputs ----
  std::vector<Event> events;
  std::map<std::string, std::string> binds;
  std::unique_ptr<Pool> pool;

  void load(const Value& in) {
    for (auto& n : in.arr_at("nodes")) node_specs.push_back(parse_node(n));
    for (auto& p : in.arr_at("pods")) pods.push_back(parse_pod(p));
    for (auto& t : in.arr_at("tiers")) {
      std::vector<PluginOpt> tier;
      for (auto& p : t.arr_at("plugins")) {
        PluginOpt o;
        o.name = p.str_at("name");
        o.job_order = p.bool_at("enabledJobOrder");
        o.job_ready = p.bool_at("enabledJobReady");
        o.job_pipelined = p.bool_at("enabledJobPipelined");
        o.task_order = p.bool_at("enabledTaskOrder");
        o.preemptable = p.bool_at("enabledPreemptable");
        o.reclaimable = p.bool_at("enabledReclaimable");
        o.queue_order = p.bool_at("enabledQueueOrder");
        o.predicate = p.bool_at("enabledPredicate");
        o.node_order = p.bool_at("enabledNodeOrder");
        const Value* a = p.get("arguments");
        if (a && a->kind == Value::Obj)
          for (auto& kv : a->o) o.args[kv.first] = kv.second.kind == Value::Str ? kv.second.s : std::to_string(kv.second.as_int());
        tier.push_back(o);
      }
      tiers.push_back(tier);
    }
    // Nodes: NewNodeInfo + AddTask for every non-terminated pod on it; Snapshot keeps Ready ones.
    std::vector<int> order(node_specs.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = (int)i;
    std::sort(order.begin(), order.end(), [&](int a, int b) { return node_specs[a].name < node_specs[b].name; });
    std::map<std::string, NodeI> all;
    for (int i : order) {
      NodeI ni;
      ni.name = node_specs[i].name;
      ni.node = &node_specs[i];
      ni.idle = Resource::from_list(node_specs[i].alloc);
      ni.alloc = Resource::from_list(node_specs[i].alloc);
      ni.cap = Resource::from_list(node_specs[i].cap);
      all[ni.name] = ni;
    }
    // Jobs (getOrCreateJob: only pods with a group annotation; shadow PodGroups are out of scope).
    for (auto& p : pods) {
      tasks.emplace_back();
      Task& t = tasks.back();
      t.uid = p.uid;
      t.name = p.name;
      t.ns = p.ns;
      t.node_name = p.node;
      t.status = get_task_status(p);
      t.priority = p.has_priority ? p.priority : 1;
      t.pod = &p;
      t.resreq = pod_resreq(p);
      t.initreq = pod_initreq(p);
      if (!p.group.empty()) {
        t.job = p.ns + "/" + p.group;  // getJobID (job_info.go:57-66)
        Job& j = jobs[t.job];
        j.uid = t.job;
        j.add_task_info(&t);
      }
      if (!p.node.empty()) {
        auto it = all.find(p.node);
        if (it == all.end()) continue;  // a node unknown to the cache never becomes Ready
        if (t.status != Succeeded && t.status != Failed) it->second.add_task(&t);
      }
    }
    for (auto& g : in.arr_at("podGroups")) {
      std::string uid = g.str_at("ns") + "/" + g.str_at("name");
      Job& j = jobs[uid];
      j.uid = uid;
      j.has_pg = true;
      j.name = g.str_at("name");
      j.ns = g.str_at("ns");
      j.min_avail = (int32_t)g.int_at("minMember");
      j.queue = g.str_at("queue");
      j.ctime = g.int_at("ctime");
      j.pg_phase = g.str_at("phase");
      j.priority = (int32_t)g.int_at("priority");
    }
    for (auto& q : in.arr_at("queues")) {
      QueueI qi;
      qi.uid = qi.name = q.str_at("name");
      qi.weight = (int32_t)q.int_at("weight", 1);
      qi.ctime = q.int_at("ctime");
      queues[qi.uid] = qi;
    }
    for (auto it = jobs.begin(); it != jobs.end();) {
      if (!it->second.has_pg || !queues.count(it->second.queue)) it = jobs.erase(it);
      else ++it;
    }
    // NodeInfo.Ready(): Used <= Allocatable (node_info.go:104-134)
    for (auto& kv : all) {
      NodeI& ni = kv.second;
      if (!ni.used.less_equal(Resource::from_list(ni.node->alloc))) continue;
      node_index[ni.name] = (int)nodes.size();
      nodes.push_back(ni);
    }
    pool.reset(new Pool(opt.workers));
    open_plugins();
  }

  // ---- tier dispatch (framework/session_plugins.go) ----
  const PluginOpt* find_opt(const std::string& n) const {
    for (auto& t : tiers)
      for (auto& p : t)
        if (p.name == n) return &p;
    return nullptr;
  }

  // OnSessionOpen of each registered plugin (framework/framework.go:30-51)
  void open_plugins() {
    static const std::set<std::string> known = {"drf", "gang", "predicates", "priority", "nodeorder",
                                                "conformance", "proportion"};
    for (auto& t : tiers)
      for (auto& p : t)
        if (known.count(p.name)) plugins.insert(p.name);
    if (plugins.count("predicates") || plugins.count("nodeorder")) {
      has_lister = true;
      // NewPodLister (plugins/util/util.go:57-82)
      for (auto& jkv : jobs)
        for (auto& skv : jkv.second.tsi) {
          if (!allocated_status(skv.first)) continue;
          for (auto& tkv : skv.second) {
            lister_tasks[tkv.first] = tkv.second;
            if (tkv.second->pod->has_affinity) lister_aff[tkv.first] = tkv.second;
          }
        }
      // GenerateNodeMapAndSlice (plugins/util/util.go:186-198)
      knodes.resize(nodes.size());
      for (size_t i = 0; i < nodes.size(); ++i) {
        knodes[i].set_node(nodes[i].node, (int)i);
        for (const Task* t : nodes[i].tasks) knodes[i].add_pod(t->pod, node_of(t->pod->node));
      }
    }
    if (const PluginOpt* o = find_opt("predicates")) {  // predicates.go:72-111
      get_bool(o->args, &mem_pressure, "predicate.MemoryPressureEnable");
      get_bool(o->args, &disk_pressure, "predicate.DiskPressureEnable");
      get_bool(o->args, &pid_pressure, "predicate.PIDPressureEnable");
    }
    if (const PluginOpt* o = find_opt("nodeorder")) {  // nodeorder.go:96-140
      get_int(o->args, &w_na, "nodeaffinity.weight");
      get_int(o->args, &w_pa, "podaffinity.weight");
      get_int(o->args, &w_lr, "leastrequested.weight");
      get_int(o->args, &w_bra, "balancedresource.weight");
    }
    if (plugins.count("drf")) {  // drf.go:60-84
      for (auto& n : nodes) drf_total.add(n.alloc);
      for (auto& jkv : jobs) {
        Resource a;
        for (auto& skv : jkv.second.tsi)
          if (allocated_status(skv.first))
            for (auto& tkv : skv.second) a.add(tkv.second->resreq);
        drf_alloc[jkv.first] = a;
        drf_share[jkv.first] = drf_calc_share(a);
      }
    }
    if (plugins.count("proportion")) open_proportion();
  }

  int node_of(const std::string& name) const {
    auto it = node_index.find(name);
    return it == node_index.end() ? -1 : it->second;
  }

  // drf.calculateShare (drf.go:161-171)
  double drf_calc_share(const Resource& a) const {
    double res = 0;
    for (auto& rn : drf_total.names()) {
      double s = share(a.get(rn), drf_total.get(rn));
      if (s > res) res = s;
    }
    return res;
  }

  // proportion.OnSessionOpen (proportion.go:58-169); queues iterated in UID order.
  void open_proportion() {
    for (auto& n : nodes) prop_total.add(n.alloc);
    for (auto& jkv : jobs) {
      Job& job = jkv.second;
      if (!prop.count(job.queue)) {
        QueueI& q = queues[job.queue];
        QAttr a;
        a.id = q.uid;
        a.name = q.name;
        a.weight = q.weight;
        prop[job.queue] = a;
      }
      QAttr& attr = prop[job.queue];
      for (auto& skv : job.tsi) {
        if (allocated_status(skv.first)) {
          for (auto& tkv : skv.second) { attr.allocated.add(tkv.second->resreq); attr.request.add(tkv.second->resreq); }
        } else if (skv.first == Pending) {
          for (auto& tkv : skv.second) attr.request.add(tkv.second->resreq);
        }
      }
    }
    Resource remaining = prop_total;
    std::set<std::string> meet;
    for (;;) {
      int32_t total_weight = 0;
      for (auto& kv : prop)
        if (!meet.count(kv.second.id)) total_weight += kv.second.weight;
      if (total_weight == 0) break;
      Resource inc, dec;
      for (auto& kv : prop) {
        QAttr& attr = kv.second;
        if (meet.count(attr.id)) continue;
        Resource old = attr.deserved;
        Resource part = remaining;
        attr.deserved.add(part.multi((double)attr.weight / (double)total_weight));
        if (attr.request.less(attr.deserved)) {
          attr.deserved = res_min(attr.deserved, attr.request);
          meet.insert(attr.id);
        }
        prop_update_share(attr);
        // Resource.Diff (resource_info.go:278-309)
        Resource i2, d2;
        if (attr.deserved.cpu > old.cpu) i2.cpu += attr.deserved.cpu - old.cpu; else d2.cpu += old.cpu - attr.deserved.cpu;
        if (attr.deserved.mem > old.mem) i2.mem += attr.deserved.mem - old.mem; else d2.mem += old.mem - attr.deserved.mem;
        for (auto& s : attr.deserved.sc) {
          double rq = old.get_sc(s.first);
          if (s.second > rq) { i2.has_map = true; i2.sc[s.first] += s.second - rq; }
          else { d2.has_map = true; d2.sc[s.first] += rq - s.second; }
        }
        inc.add(i2);
        dec.add(d2);
      }
      remaining.sub(inc).add(dec);
      if (remaining.is_empty()) break;
    }
  }
  // proportion.updateShare (proportion.go:265-277)
  void prop_update_share(QAttr& attr) {
    double res = 0;
    for (auto& rn : attr.deserved.names()) {
      double s = share(attr.allocated.get(rn), attr.deserved.get(rn));
      if (s > res) res = s;
    }
    attr.share = res;
  }

  // ---- order fns ----
  // JobOrderFn (session_plugins.go:281-305)
  bool job_less(const Job* l, const Job* r) const {
    for (auto& tier : tiers)
      for (auto& p : tier) {
        if (!p.job_order || !plugins.count(p.name)) continue;
        int j = 0;
        if (p.name == "priority") j = l->priority > r->priority ? -1 : (l->priority < r->priority ? 1 : 0);  // priority.go:60-78
        else if (p.name == "gang") {  // gang.go:96-119
          bool lr = l->ready(), rr = r->ready();
          j = (lr && rr) ? 0 : lr ? 1 : rr ? -1 : 0;
        } else if (p.name == "drf") {  // drf.go:114-130
          double ls = drf_share.at(l->uid), rs = drf_share.at(r->uid);
          j = ls == rs ? 0 : (ls < rs ? -1 : 1);
        } else continue;
        if (j != 0) return j < 0;
      }
    if (l->ctime == r->ctime) return l->uid < r->uid;
    return l->ctime < r->ctime;
  }
  // QueueOrderFn (session_plugins.go:308-333)
  bool queue_less(const QueueI* l, const QueueI* r) const {
    for (auto& tier : tiers)
      for (auto& p : tier) {
        if (!p.queue_order || !plugins.count(p.name)) continue;
        if (p.name != "proportion") continue;
        double ls = prop.at(l->uid).share, rs = prop.at(r->uid).share;  // proportion.go:171-184
        int j = ls == rs ? 0 : (ls < rs ? -1 : 1);
        if (j != 0) return j < 0;
      }
    if (l->ctime == r->ctime) return l->uid < r->uid;
    return l->ctime < r->ctime;
  }
  // TaskOrderFn (session_plugins.go:336-369)
  bool task_less(const Task* l, const Task* r) const {
    for (auto& tier : tiers)
      for (auto& p : tier) {
        if (!p.task_order || !plugins.count(p.name)) continue;
        if (p.name != "priority") continue;
        int j = l->priority == r->priority ? 0 : (l->priority > r->priority ? -1 : 1);  // priority.go:40-56
        if (j != 0) return j < 0;
      }
    if (l->pod->ctime == r->pod->ctime) return l->uid < r->uid;
    return l->pod->ctime < r->pod->ctime;
  }
  // JobValid (session_plugins.go:243-259) -- gang.go:48-69
  bool job_valid(const Job* j) const {
    for (auto& tier : tiers)
      for (auto& p : tier)
        if (p.name == "gang" && plugins.count("gang") && j->valid_task_num() < j->min_avail) return false;
    return true;
  }
  // JobReady (session_plugins.go:202-220) -- gang.go:122-125
  bool job_ready(const Job* j) const {
    for (auto& tier : tiers)
      for (auto& p : tier)
        if (p.job_ready && p.name == "gang" && plugins.count("gang") && !j->ready()) return false;
    return true;
  }
  // Overused (session_plugins.go:185-199) -- proportion.go:221-233
  bool overused(const QueueI* q) const {
    for (auto& tier : tiers)
      for (auto& p : tier)
        if (p.name == "proportion" && plugins.count("proportion")) {
          const QAttr& a = prop.at(q->uid);
          if (a.deserved.less_equal(a.allocated)) return true;
        }
    return false;
  }
  bool predicate_enabled() const {
    for (auto& tier : tiers)
      for (auto& p : tier)
        if (p.predicate && p.name == "predicates" && plugins.count("predicates")) return true;
    return false;
  }
  bool nodeorder_enabled() const {
    for (auto& tier : tiers)
      for (auto& p : tier)
        if (p.node_order && p.name == "nodeorder" && plugins.count("nodeorder")) return true;
    return false;
  }

  // ---- predicates plugin closure (plugins/predicates/predicates.go:154-299) ----
  PredResult predicates_fn(const Task* task, int ni) const {
    const KNode& kn = knodes[ni];
    const NodeI& node = nodes[ni];
    const Pod& pod = *task->pod;
    const NodeSpec& ns = *node.node;
    // pod number (:162-166)
    if (node.alloc.max_task <= (int)kn.pods.size()) return PredResult::fail({kPodNumberExceeded});
    // CheckNodeConditionPredicate (vendor/.../predicates.go:1568-1596)
    {
      std::vector<std::string> r;
      for (auto& c : ns.conditions) {
        if (c.first == "Ready" && c.second != "True") r.push_back(kNodeNotReady);
        else if (c.first == "OutOfDisk" && c.second != "False") r.push_back(kNodeOutOfDisk);
        else if (c.first == "NetworkUnavailable" && c.second != "False") r.push_back(kNodeNetworkUnavailable);
      }
      if (ns.unschedulable) r.push_back(kNodeUnschedulable);
      if (!r.empty()) return PredResult::fail(r);
    }
    // CheckNodeUnschedulablePredicate (:1469-1487)
    if (ns.unschedulable) {
      bool tol = false;
      for (auto& t : pod.tolerations)
        if (tolerates(t, {"node.kubernetes.io/unschedulable", "", "NoSchedule"})) tol = true;
      if (!tol) return PredResult::fail({kNodeUnschedulable});
    }
    // PodMatchNodeSelector (:853-863, :807-850)
    if (!pod_matches_node_selector_and_affinity(pod, ns)) return PredResult::fail({kNodeSelectorNotMatch});
    // PodFitsHostPorts (:1031-1052); GetContainerPorts: containers only (scheduler/util/utils.go:30-41)
    for (auto& c : pod.containers)
      for (auto& pt : c.ports)
        if (kn.check_conflict(pt.host_ip, pt.protocol, pt.host_port)) return PredResult::fail({kHostPorts});
    // PodToleratesNodeTaints (:1489-1518)
    for (auto& t : ns.taints) {
      if (t.effect != "NoSchedule" && t.effect != "NoExecute") continue;
      bool tol = false;
      for (auto& o : pod.tolerations)
        if (tolerates(o, t)) { tol = true; break; }
      if (!tol) return PredResult::fail({kTaints});
    }
    // pressure predicates (:233-276; vendored :1526-1566)
    if (mem_pressure && is_best_effort(pod) && kn.mem_pressure == "True") return PredResult::fail({kMemPressure});
    if (disk_pressure && kn.disk_pressure == "True") return PredResult::fail({kDiskPressure});
    if (pid_pressure && kn.pid_pressure == "True") return PredResult::fail({kPIDPressure});
    // inter-pod affinity (:278-296)
    return interpod_affinity_matches(task, ni);
  }

  // Toleration.ToleratesTaint (vendor/k8s.io/api/core/v1/toleration.go:37-56)
  static bool tolerates(const Toleration& t, const Taint& taint) {
    if (!t.effect.empty() && t.effect != taint.effect) return false;
    if (!t.key.empty() && t.key != taint.key) return false;
    if (t.op.empty() || t.op == "Equal") return t.value == taint.value;
    if (t.op == "Exists") return true;
    return false;
  }
  // v1qos.GetPodQOS == BestEffort: no container or init container requests/limits of cpu or memory.
  static bool is_best_effort(const Pod& p) {
    auto has = [](const std::vector<Container>& cs) {
      for (auto& c : cs)
        if (c.req.get("cpu") || c.req.get("memory")) return true;
      return false;
    };
    return !has(p.containers) && !has(p.init);
  }
  // podMatchesNodeSelectorAndAffinityTerms (vendor/.../predicates.go:807-850)
  static bool pod_matches_node_selector_and_affinity(const Pod& pod, const NodeSpec& node) {
    if (!pod.node_selector.empty()) {
      if (!selector_from_set(pod.node_selector).matches(node.labels)) return false;
    }
    if (pod.has_affinity && pod.aff.has_node) {
      if (!pod.aff.node.has_required) return true;
      return match_node_selector_terms(pod.aff.node.required, node.labels, node.name);
    }
    return true;
  }

  // ---- inter-pod affinity predicate (vendor/.../predicates.go:1155-1465) ----
  struct PodMatch {  // affinityTermProperties (metadata.go:310-345)
    std::set<std::string> namespaces;
    Selector sel;
  };
  static std::set<std::string> term_namespaces(const Pod& owner, const PodAffinityTerm& t) {  // topologies.go:28-38
    std::set<std::string> s;
    if (t.namespaces.empty()) s.insert(owner.ns);
    else s.insert(t.namespaces.begin(), t.namespaces.end());
    return s;
  }
  static bool pod_matches_ns_sel(const Pod& p, const std::set<std::string>& nss, const Selector& sel) {  // topologies.go:42-51
    return nss.count(p.ns) && sel.matches(p.labels);
  }
  // NodesHaveSameTopologyKey (priorities/util/topologies.go:53-71)
  static bool same_topology(const NodeSpec* a, const NodeSpec* b, const std::string& key) {
    if (key.empty()) return false;
    auto ia = a->labels.find(key), ib = b->labels.find(key);
    if (ia == a->labels.end() || ib == b->labels.end()) return false;
    return ia->second == ib->second;
  }

  // The lister list the predicate sees: FilteredList(nodeInfo.Filter, Everything()) over the affinity
  // lister when the incoming pod has no affinity (predicates.go:279-283; plugins/util/util.go:153-176).
  std::vector<const Task*> lister_list(const Task* task, int ni) const {
    const auto& set = task->pod->has_affinity ? lister_tasks : lister_aff;
    std::vector<const Task*> out;
    out.reserve(set.size());
    for (auto& kv : set) {
      const Task* t = kv.second;
      // NodeInfo.Filter (cache/node_info.go:692-702)
      if (t->node_name == nodes[ni].name) {
        bool found = false;
        for (auto& pr : knodes[ni].pods)
          if (pr.pod->name == t->pod->name && pr.pod->ns == t->pod->ns) { found = true; break; }
        if (!found) continue;
      }
      out.push_back(t);
    }
    return out;
  }

  PredResult interpod_affinity_matches(const Task* task, int ni) const {
    if (opt.literal_affinity) return interpod_affinity_literal(task, ni);
    return interpod_affinity_fast(task, ni);
  }

  // Literal restatement of the meta == nil slow path (predicates.go:1155-1185, 1293-1333, 1367-1465).
  PredResult interpod_affinity_literal(const Task* task, int ni) const {
    const Pod& pod = *task->pod;
    const NodeSpec* node = nodes[ni].node;
    std::vector<const Task*> filtered = lister_list(task, ni);
    // satisfiesExistingPodsAntiAffinity (:1293-1333) via getMatchingAntiAffinityTopologyPairsOfPods (:1247-1291)
    std::set<std::pair<std::string, std::string>> pairs;
    // errors come back as FitErrors.SetNodeError(err): the error's own string, no reason constants
    const std::string pn = pod.ns + "/" + pod.name;  // podName (vendor/.../predicates.go:721-723)
    for (const Task* et : filtered) {
      int en = node_of(et->node_name);
      if (en < 0)
        return PredResult::fail({"Failed to get all terms that pod " + pn + " matches, err: failed to find node <" +
                                 et->node_name + ">"});
      const Pod& ep = *et->pod;
      if (!ep.has_affinity || !ep.aff.has_anti) continue;
      for (auto& term : ep.aff.anti.required) {
        Selector sel;
        std::string err;
        if (!label_selector_as_selector(term.sel, &sel, &err))
          return PredResult::fail({"Failed to get all terms that pod " + pn + " matches, err: " + err});
        if (pod_matches_ns_sel(pod, term_namespaces(ep, term), sel)) {
          auto it = nodes[en].node->labels.find(term.topology_key);
          if (it != nodes[en].node->labels.end()) pairs.insert({term.topology_key, it->second});
        }
      }
    }
    for (auto& kv : node->labels)
      if (pairs.count(kv)) return PredResult::fail({kPodAffinityNotMatch, kExistingAntiAffinity});
    if (!pod.has_affinity || (!pod.aff.has_pod && !pod.aff.has_anti)) return PredResult();
    // satisfiesPodsAffinityAntiAffinity slow path (:1401-1457)
    const auto& aff_terms = pod.aff.has_pod ? pod.aff.pod.required : empty_terms();
    const auto& anti_terms = pod.aff.has_anti ? pod.aff.anti.required : empty_terms();
    bool match_found = false, sel_found = false;
    for (const Task* tt : filtered) {
      if (!match_found && !aff_terms.empty()) {
        bool all, props;
        std::string err;
        if (!pod_matches_terms(pod, tt, ni, aff_terms, &all, &props, &err))
          return PredResult::fail({"Cannot schedule pod " + pn + " onto node " + node->name +
                                   ", because of PodAffinity, err: " + err});
        if (props) sel_found = true;
        if (all) match_found = true;
      }
      if (!anti_terms.empty()) {
        bool all, props;
        std::string err;
        bool ok = pod_matches_terms(pod, tt, ni, anti_terms, &all, &props, &err);
        if (!ok || all) return PredResult::fail({kPodAffinityNotMatch, kPodAntiAffinityRules});
      }
    }
    if (!match_found && !aff_terms.empty()) {
      if (sel_found) return PredResult::fail({kPodAffinityNotMatch, kPodAffinityRules});
      if (!target_matches_affinity_of_pod(pod, pod)) return PredResult::fail({kPodAffinityNotMatch, kPodAffinityRules});
    }
    return PredResult();
  }
  static const std::vector<PodAffinityTerm>& empty_terms() {
    static const std::vector<PodAffinityTerm> e;
    return e;
  }
  // podMatchesPodAffinityTerms (:1189-1214)
  bool pod_matches_terms(const Pod& pod, const Task* target, int ni, const std::vector<PodAffinityTerm>& terms,
                         bool* all, bool* props_ok, std::string* err) const {
    *all = *props_ok = false;
    // getAffinityTermProperties (metadata.go:317-331) builds every term's selector first
    std::vector<Selector> sels(terms.size());
    for (size_t i = 0; i < terms.size(); ++i)
      if (!label_selector_as_selector(terms[i].sel, &sels[i], err)) return false;
    for (size_t i = 0; i < terms.size(); ++i)  // podMatchesAllAffinityTermProperties (:334-345)
      if (!pod_matches_ns_sel(*target->pod, term_namespaces(pod, terms[i]), sels[i])) return true;
    int tn = node_of(target->node_name);
    if (tn < 0) { *err = "failed to find node <" + target->node_name + ">"; return false; }
    for (auto& t : terms) {
      if (t.topology_key.empty()) {
        *err = "empty topologyKey is not allowed except for PreferredDuringScheduling pod anti-affinity";
        return false;
      }
      if (!same_topology(nodes[ni].node, nodes[tn].node, t.topology_key)) { *props_ok = true; return true; }
    }
    *all = *props_ok = true;
    return true;
  }
  // targetPodMatchesAffinityOfPod (metadata.go:498-510)
  static bool target_matches_affinity_of_pod(const Pod& pod, const Pod& target) {
    if (!pod.has_affinity || !pod.aff.has_pod) return false;
    const auto& terms = pod.aff.pod.required;
    if (terms.empty()) return false;
    for (auto& t : terms) {
      Selector sel;
      if (!label_selector_as_selector(t.sel, &sel)) return false;
      if (!pod_matches_ns_sel(target, term_namespaces(pod, t), sel)) return false;
    }
    return true;
  }

  // Per-task precomputed form of the same predicate: the lister scan is hoisted out of the node
  // loop (what predicateMetadata does in metadata.go:115-165). Equal to the literal form when every
  // lister pod sits on a session node and no selector is invalid (checked by tests).
  struct AffPre {
    bool built = false;
    std::set<std::pair<std::string, std::string>> anti_pairs;
    bool has_aff = false, has_anti = false, sel_found = false, self_match = false;
    std::set<std::vector<std::string>> aff_tuples, anti_tuples;
    std::vector<std::string> aff_keys, anti_keys;
    std::string error;
  };
  mutable std::map<const Task*, AffPre> aff_cache;
  mutable std::mutex aff_mu;
  mutable uint64_t aff_epoch = 0, aff_cache_epoch = ~0ULL;

  const AffPre& aff_pre(const Task* task) const {
    std::lock_guard<std::mutex> g(aff_mu);
    if (aff_cache_epoch != aff_epoch) { aff_cache.clear(); aff_cache_epoch = aff_epoch; }
    AffPre& a = aff_cache[task];
    if (a.built) return a;
    a.built = true;
    const Pod& pod = *task->pod;
    const auto& set = pod.has_affinity ? lister_tasks : lister_aff;
    for (auto& kv : set) {
      const Task* et = kv.second;
      int en = node_of(et->node_name);
      if (en < 0) { a.error = "failed to find node <" + et->node_name + ">"; return a; }
      const Pod& ep = *et->pod;
      if (!ep.has_affinity || !ep.aff.has_anti) continue;
      for (auto& term : ep.aff.anti.required) {
        Selector sel;
        if (!label_selector_as_selector(term.sel, &sel)) { a.error = "invalid label selector"; return a; }
        if (pod_matches_ns_sel(pod, term_namespaces(ep, term), sel)) {
          auto it = nodes[en].node->labels.find(term.topology_key);
          if (it != nodes[en].node->labels.end()) a.anti_pairs.insert({term.topology_key, it->second});
        }
      }
    }
    if (!pod.has_affinity) return a;
    auto collect = [&](const std::vector<PodAffinityTerm>& terms, std::set<std::vector<std::string>>* tuples,
                       std::vector<std::string>* keys, bool* any_props) -> bool {
      std::vector<std::pair<std::set<std::string>, Selector>> props;
      for (auto& t : terms) {
        Selector sel;
        if (!label_selector_as_selector(t.sel, &sel)) return false;
        props.emplace_back(term_namespaces(pod, t), sel);
        keys->push_back(t.topology_key);
      }
      for (auto& kv : set) {
        const Task* tt = kv.second;
        bool m = true;
        for (auto& p : props)
          if (!pod_matches_ns_sel(*tt->pod, p.first, p.second)) { m = false; break; }
        if (!m) continue;
        if (any_props) *any_props = true;
        for (auto& k : *keys)
          if (k.empty()) return false;
        const NodeSpec* tn = nodes[node_of(tt->node_name)].node;
        std::vector<std::string> tup;
        bool ok = true;
        for (auto& k : *keys) {
          auto it = tn->labels.find(k);
          if (it == tn->labels.end()) { ok = false; break; }
          tup.push_back(it->second);
        }
        if (ok) tuples->insert(tup);
      }
      return true;
    };
    if (pod.aff.has_pod && !pod.aff.pod.required.empty()) {
      a.has_aff = true;
      if (!collect(pod.aff.pod.required, &a.aff_tuples, &a.aff_keys, &a.sel_found)) { a.error = "affinity"; return a; }
      a.self_match = target_matches_affinity_of_pod(pod, pod);
    }
    if (pod.aff.has_anti && !pod.aff.anti.required.empty()) {
      a.has_anti = true;
      if (!collect(pod.aff.anti.required, &a.anti_tuples, &a.anti_keys, nullptr)) { a.error = "anti-affinity"; return a; }
    }
    return a;
  }
  mutable const AffPre* sweep_aff = nullptr;  // set for the duration of one PredicateNodes sweep
  PredResult interpod_affinity_fast(const Task* task, int ni) const {
    const AffPre& a = sweep_aff ? *sweep_aff : aff_pre(task);
    if (!a.error.empty()) return interpod_affinity_literal(task, ni);
    const NodeSpec* node = nodes[ni].node;
    for (auto& kv : node->labels)
      if (a.anti_pairs.count(kv)) return PredResult::fail({kPodAffinityNotMatch, kExistingAntiAffinity});
    auto tuple_of = [&](const std::vector<std::string>& keys, std::vector<std::string>* tup) {
      for (auto& k : keys) {
        auto it = node->labels.find(k);
        if (it == node->labels.end()) return false;
        tup->push_back(it->second);
      }
      return true;
    };
    if (a.has_anti) {
      std::vector<std::string> tup;
      if (tuple_of(a.anti_keys, &tup) && a.anti_tuples.count(tup))
        return PredResult::fail({kPodAffinityNotMatch, kPodAntiAffinityRules});
    }
    if (a.has_aff) {
      std::vector<std::string> tup;
      bool match = tuple_of(a.aff_keys, &tup) && a.aff_tuples.count(tup);
      if (!match && (a.sel_found || !a.self_match)) return PredResult::fail({kPodAffinityNotMatch, kPodAffinityRules});
    }
    return PredResult();
  }

  // ---- allocate's predicateFn closure (actions/allocate/allocate.go:80-93) + Session.PredicateFn ----
  PredResult alloc_predicate(const Task* task, int ni) const {
    const NodeI& n = nodes[ni];
    if (!task->initreq.less_equal(n.idle) && !task->initreq.less_equal(n.releasing))
      return PredResult::fail({kResourceFit});
    // Session.PredicateFn (session_plugins.go:372-389): only the predicates plugin registers one.
    if (predicate_enabled()) return predicates_fn(task, ni);
    return PredResult();
  }

  // ---- nodeorder (plugins/nodeorder/nodeorder.go:188-246) ----
  // LeastRequestedPriorityMap / BalancedResourceAllocationMap (priorities/least_requested.go:33-53,
  // balanced_resource_allocation.go:38-77, resource_allocation.go:39-103)
  static int64_t lr_score(int64_t req, int64_t cap) {
    if (cap == 0) return 0;
    if (req > cap) return 0;
    return ((cap - req) * 10) / cap;
  }
  static double fraction(int64_t req, int64_t cap) {
    if (cap == 0) return 1;
    return (double)req / (double)cap;
  }
  void task_nonzero(const Task* t, int64_t* cpu, int64_t* mem) const {
    *cpu = *mem = 0;
    for (auto& c : t->pod->containers) {
      int64_t a, b;
      nonzero_requests(c.req, &a, &b);
      *cpu += a;
      *mem += b;
    }
  }
  // returns false when the map fn errors (CalculateNodeAffinityPriorityMap on an invalid term)
  bool node_order_fn(const Task* task, int ni, double* score) const {
    const KNode& kn = knodes[ni];
    int64_t rc, rm;
    task_nonzero(task, &rc, &rm);
    rc += kn.nz_cpu;
    rm += kn.nz_mem;
    int64_t lr = (lr_score(rc, kn.alloc_cpu) + lr_score(rm, kn.alloc_mem)) / 2;
    double cf = fraction(rc, kn.alloc_cpu), mf = fraction(rm, kn.alloc_mem);
    int64_t bra = (cf >= 1 || mf >= 1) ? 0 : (int64_t)((1 - std::fabs(cf - mf)) * 10);
    // CalculateNodeAffinityPriorityMap (priorities/node_affinity.go:34-74)
    int32_t count = 0;
    const Pod& pod = *task->pod;
    if (pod.has_affinity && pod.aff.has_node) {
      for (auto& pt : pod.aff.node.preferred) {
        if (pt.first == 0) continue;
        Selector s;
        if (!node_reqs_as_selector(pt.second.exprs, &s)) return false;
        if (s.matches(kn.node->labels)) count += pt.first;
      }
    }
    double sc = 0.0;
    sc = sc + (double)(lr * (int64_t)w_lr);
    sc = sc + (double)(bra * (int64_t)w_bra);
    sc = sc + (double)((int64_t)count * (int64_t)w_na);
    *score = sc;
    return true;
  }

  // ---- CalculateInterPodAffinityPriority (priorities/interpod_affinity.go:119-241) ----
  // Histogram form: counts[n] = sum_k hist_k[label_k(n)], equal to the literal per-node loop of
  // processTerm (:86-103) because every increment is an integer (exact in float64).
  bool ipa_scores(const Task* task, std::vector<double>* out) const {
    const Pod& pod = *task->pod;
    bool has_aff = pod.has_affinity && pod.aff.has_pod;
    bool has_anti = pod.has_affinity && pod.aff.has_anti;
    std::map<std::string, std::map<std::string, double>> hist;
    std::vector<double> lit;
    if (opt.literal_affinity) lit.assign(nodes.size(), 0.0);
    bool err = false;
    auto process_term = [&](const PodAffinityTerm& term, const Pod& definer, const Pod& to_check, int fixed,
                            double w) {
      Selector sel;
      if (!label_selector_as_selector(term.sel, &sel)) { err = true; return; }
      if (!pod_matches_ns_sel(to_check, term_namespaces(definer, term), sel)) return;
      if (opt.literal_affinity) {
        for (size_t n = 0; n < nodes.size(); ++n)
          if (same_topology(nodes[n].node, nodes[fixed].node, term.topology_key)) lit[n] += w;
        return;
      }
      if (term.topology_key.empty()) return;
      auto it = nodes[fixed].node->labels.find(term.topology_key);
      if (it == nodes[fixed].node->labels.end()) return;
      hist[term.topology_key][it->second] += w;
    };
    auto process_pod = [&](const PodRef& e) {
      if (e.node < 0) return;  // GetNodeInfo miss (cachedNodeInfo fallback is out of scope)
      const Pod& ep = *e.pod;
      if (has_aff)
        for (auto& t : pod.aff.pod.preferred) process_term(t.term, pod, ep, e.node, (double)(t.weight * 1));
      if (has_anti)
        for (auto& t : pod.aff.anti.preferred) process_term(t.term, pod, ep, e.node, (double)(t.weight * -1));
      if (ep.has_affinity && ep.aff.has_pod) {
        for (auto& t : ep.aff.pod.required) process_term(t, ep, pod, e.node, 1.0);  // hardPodAffinityWeight = 1
        for (auto& t : ep.aff.pod.preferred) process_term(t.term, ep, pod, e.node, (double)(t.weight * 1));
      }
      if (ep.has_affinity && ep.aff.has_anti)
        for (auto& t : ep.aff.anti.preferred) process_term(t.term, ep, pod, e.node, (double)(t.weight * -1));
    };
    for (size_t n = 0; n < knodes.size(); ++n) {
      const auto& list = (has_aff || has_anti) ? knodes[n].pods : knodes[n].pods_with_affinity;
      for (auto& e : list) process_pod(e);
    }
    if (err) return false;
    std::vector<double>& counts = *out;
    counts.assign(nodes.size(), 0.0);
    for (size_t n = 0; n < nodes.size(); ++n) {
      if (opt.literal_affinity) { counts[n] = lit[n]; continue; }
      double c = 0;
      for (auto& hk : hist) {
        auto it = nodes[n].node->labels.find(hk.first);
        if (it == nodes[n].node->labels.end()) continue;
        auto hv = hk.second.find(it->second);
        if (hv != hk.second.end()) c += hv->second;
      }
      counts[n] = c;
    }
    double maxc = 0, minc = 0;
    for (double c : counts) {
      if (c > maxc) maxc = c;
      if (c < minc) minc = c;
    }
    for (size_t n = 0; n < nodes.size(); ++n) {
      double f = 0;
      if ((maxc - minc) > 0) f = 10.0 * ((counts[n] - minc) / (maxc - minc));
      counts[n] = (double)(int64_t)f;  // HostPriority.Score = int(fScore)
    }
    return true;
  }

  // ---- util.PredicateNodes / PrioritizeNodes / SelectBestNode (util/scheduler_helper.go:34-158) ----
  struct Sweep {
    std::vector<PredResult> pred;
    std::vector<int> feasible;
    std::vector<double> score;    // per feasible position
    bool batch_error = false;
  };
  void predicate_nodes(const Task* task, Sweep* s) const {
    s->pred.assign(nodes.size(), PredResult());
    sweep_aff = &aff_pre(task);  // the per-task lister scan, hoisted out of the node loop
    pool->run((int)nodes.size(), [&](int i) { s->pred[i] = alloc_predicate(task, i); });
    sweep_aff = nullptr;
    s->feasible.clear();
    for (size_t i = 0; i < nodes.size(); ++i)
      if (s->pred[i].ok) s->feasible.push_back((int)i);
  }
  void prioritize_nodes(const Task* task, Sweep* s) const {
    const std::vector<int>& f = s->feasible;
    std::vector<double> order(f.size(), 0.0);
    std::vector<char> have(f.size(), 0);
    bool no = nodeorder_enabled();
    pool->run((int)f.size(), [&](int i) {
      // Session.NodeOrderMapFn (session_plugins.go:443-469)
      double sc = 0;
      if (no) {
        double v;
        if (!node_order_fn(task, f[i], &v)) return;  // error: node left out of nodeOrderScoreMap
        sc = sc + v;
      }
      order[i] = sc;
      have[i] = 1;
    });
    std::vector<double> batch;
    bool have_batch = false;
    if (no) {  // Session.BatchNodeOrderFn (session_plugins.go:415-436) -> nodeorder.go:229-246
      if (!ipa_scores(task, &batch)) { s->batch_error = true; return; }
      for (auto& b : batch) b = b * (double)w_pa;
      have_batch = true;
    }
    s->score.assign(f.size(), 0.0);
    for (size_t i = 0; i < f.size(); ++i) {
      double score = 0.0;
      if (have[i]) score = score + order[i];
      if (have_batch) score = score + (0.0 + batch[f[i]]);
      s->score[i] = score;
    }
  }
  // preempt's sweep (actions/preempt/preempt.go:187-195): PredicateNodes with ssn.PredicateFn alone (the
  // allocate closure's resource check is not part of it), PrioritizeNodes, SortNodes (util/scheduler_helper.go:
  // 132-144): scores descending, a bucket's nodes in canonical order (the reference appends them in goroutine
  // completion order). A batch-score error leaves no scores, so no nodes.
  std::vector<std::pair<int, double>> sort_nodes(const Task* task, Sweep* sw = nullptr) const {
    Sweep local;
    Sweep& s = sw ? *sw : local;
    s.pred.assign(nodes.size(), PredResult());
    sweep_aff = &aff_pre(task);
    const bool pe = predicate_enabled();
    pool->run((int)nodes.size(), [&](int i) { s.pred[i] = pe ? predicates_fn(task, i) : PredResult(); });
    sweep_aff = nullptr;
    for (size_t i = 0; i < nodes.size(); ++i)
      if (s.pred[i].ok) s.feasible.push_back((int)i);
    std::vector<std::pair<int, double>> out;
    if (s.feasible.empty()) return out;
    prioritize_nodes(task, &s);
    if (s.batch_error) return out;
    for (size_t i = 0; i < s.feasible.size(); ++i) out.emplace_back(s.feasible[i], s.score[i]);
    std::stable_sort(out.begin(), out.end(), [](const std::pair<int, double>& a, const std::pair<int, double>& b) {
      return a.second > b.second;  // sort.Reverse(sort.Float64Slice(keys)); feasible is in index order
    });
    return out;
  }

  // SelectBestNode with the lowest-index tie-break; -1 where the reference panics.
  static int select_best(const Sweep& s) {
    double max_score = -1.0;
    int best = -1;
    for (size_t i = 0; i < s.feasible.size(); ++i)
      if (s.score[i] > max_score) { max_score = s.score[i]; best = s.feasible[i]; }
    return best;
  }

  // ---- commit: Session.Allocate / Session.Pipeline (framework/session.go:199-297) ----
  void on_allocate_event(Task* task) {
    int ni = node_of(task->node_name);
    if (has_lister) {
      // PodLister.UpdateTask (plugins/util/util.go:108-130)
      if (!allocated_status(task->status)) {
        lister_tasks.erase(task->uid);
        if (task->pod->has_affinity) lister_aff.erase(task->uid);
      } else {
        lister_tasks[task->uid] = task;
        if (task->pod->has_affinity) lister_aff[task->uid] = task;
      }
      knodes[ni].add_pod(task->pod, ni);  // predicates.go:121-133 / nodeorder.go:161-172
      aff_epoch++;
    }
    if (plugins.count("drf")) {  // drf.go:135-144
      drf_alloc[task->job].add(task->resreq);
      drf_share[task->job] = drf_calc_share(drf_alloc[task->job]);
    }
    if (plugins.count("proportion")) {  // proportion.go:236-246
      QAttr& a = prop[jobs[task->job].queue];
      a.allocated.add(task->resreq);
      prop_update_share(a);
    }
  }
  void pipeline(Task* task, int ni) {
    Job& job = jobs[task->job];
    job.update_task_status(task, Pipelined);
    task->node_name = nodes[ni].name;
    nodes[ni].add_task(task);
    events.push_back({task->uid, nodes[ni].name, Pipelined});
    on_allocate_event(task);
  }
  void allocate_task(Task* task, int ni) {
    Job& job = jobs[task->job];
    job.update_task_status(task, Allocated);
    task->node_name = nodes[ni].name;
    nodes[ni].add_task(task);
    events.push_back({task->uid, nodes[ni].name, Allocated});
    on_allocate_event(task);
    if (job_ready(&job)) {  // dispatch (session.go:286-323)
      auto it = job.tsi.find(Allocated);
      if (it != job.tsi.end()) {
        std::vector<Task*> ts;
        for (auto& kv : it->second) ts.push_back(kv.second);
        for (Task* t : ts) {
          binds[t->ns + "/" + t->name] = t->node_name;
          job.update_task_status(t, Binding);
        }
      }
    }
  }

  // Go container/heap (Go 1.11 src/container/heap/heap.go) over a lessFn.
  template <class T>
  struct GoHeap {
    std::vector<T> items;
    std::function<bool(const T&, const T&)> less;
    void up(int j) {
      for (;;) {
        int i = (j - 1) / 2;
        if (i == j || !less(items[j], items[i])) break;
        std::swap(items[i], items[j]);
        j = i;
      }
    }
    void down(int i, int n) {
      for (;;) {
        int j1 = 2 * i + 1;
        if (j1 >= n || j1 < 0) break;
        int j = j1;
        int j2 = j1 + 1;
        if (j2 < n && less(items[j2], items[j1])) j = j2;
        if (!less(items[j], items[i])) break;
        std::swap(items[i], items[j]);
        i = j;
      }
    }
    void push(T x) { items.push_back(x); up((int)items.size() - 1); }
    T pop() {
      int n = (int)items.size() - 1;
      std::swap(items[0], items[n]);
      down(0, n);
      T x = items.back();
      items.pop_back();
      return x;
    }
    bool empty() const { return items.empty(); }
  };

  int64_t attempts = 0;
  double elapsed_ms = 0;
  std::string error;

  // ---- allocateAction.Execute (actions/allocate/allocate.go:42-193) ----
  void allocate() {
    auto t0 = std::chrono::steady_clock::now();
    GoHeap<QueueI*> qheap;
    qheap.less = [this](QueueI* const& a, QueueI* const& b) { return queue_less(a, b); };
    std::map<std::string, GoHeap<Job*>> jobs_map;
    for (auto& jkv : jobs) {
      Job& job = jkv.second;
      if (job.pg_phase == "Pending") continue;
      if (!job_valid(&job)) continue;
      auto q = queues.find(job.queue);
      if (q == queues.end()) continue;
      qheap.push(&q->second);
      if (!jobs_map.count(job.queue)) {
        jobs_map[job.queue].less = [this](Job* const& a, Job* const& b) { return job_less(a, b); };
      }
      jobs_map[job.queue].push(&job);
    }
    std::map<std::string, GoHeap<Task*>> pending;
    Sweep sw;
    bool stop = false;
    while (!qheap.empty() && !stop) {
      QueueI* queue = qheap.pop();
      if (overused(queue)) continue;
      auto jit = jobs_map.find(queue->uid);
      if (jit == jobs_map.end() || jit->second.empty()) continue;
      Job* job = jit->second.pop();
      if (!pending.count(job->uid)) {
        GoHeap<Task*> th;
        th.less = [this](Task* const& a, Task* const& b) { return task_less(a, b); };
        auto pit = job->tsi.find(Pending);
        if (pit != job->tsi.end())
          for (auto& kv : pit->second) {
            if (kv.second->resreq.is_empty()) continue;  // BestEffort (:116-122)
            th.push(kv.second);
          }
        pending[job->uid] = std::move(th);
      }
      GoHeap<Task*>& th = pending[job->uid];
      while (!th.empty()) {
        if (opt.max_tasks >= 0 && attempts >= opt.max_tasks) { stop = true; break; }
        Task* task = th.pop();
        attempts++;
        predicate_nodes(task, &sw);
        if (sw.feasible.empty()) {
          FitErrs fe;
          for (auto& p : sw.pred)
            if (!p.ok)
              for (auto& r : p.reasons) fe.hist[r]++;
          job->fit_errors[task->uid] = fe;
          break;
        }
        prioritize_nodes(task, &sw);
        if (sw.batch_error) { error = "panic: SelectBestNode on empty scores (batch node order error)"; stop = true; break; }
        int best = select_best(sw);
        if (best < 0) { error = "panic: SelectBestNode found no node with score > -1"; stop = true; break; }
        if (task->initreq.less_equal(nodes[best].idle)) {
          allocate_task(task, best);
        } else if (task->initreq.less_equal(nodes[best].releasing)) {
          pipeline(task, best);
        }
        if (job_ready(job)) {
          jit->second.push(job);
          break;
        }
      }
      qheap.push(queue);
    }
    elapsed_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }

  // ---- backfillAction.Execute (actions/backfill/backfill.go:40-90) ----
  // Jobs and their Pending tasks in UID order (the maps of :45 and :54), nodes in the canonical order (:62):
  // a task with an empty InitResreq takes the first node that passes Session.PredicateFn and is allocated
  // there (:71); a task that passes nowhere records its FitErrors histogram (:84-86). Other tasks are left
  // alone (:87-89).
  std::map<std::string, std::map<std::string, FitErrs>> backfill_fit_errors;
  void backfill() {
    for (auto& jkv : jobs) {
      Job& job = jkv.second;
      if (job.pg_phase == "Pending") continue;
      if (!job_valid(&job)) continue;
      auto pit = job.tsi.find(Pending);
      if (pit == job.tsi.end()) continue;
      std::vector<Task*> ts;  // allocate_task moves tasks out of the Pending index while we walk it
      for (auto& kv : pit->second) ts.push_back(kv.second);
      for (Task* task : ts) {
        if (!task->initreq.is_empty()) continue;
        FitErrs fe;
        bool allocated = false;
        for (size_t ni = 0; ni < nodes.size(); ++ni) {
          PredResult p = predicate_enabled() ? predicates_fn(task, (int)ni) : PredResult();
          if (!p.ok) {
            for (auto& r : p.reasons) fe.hist[r]++;
            continue;
          }
          allocate_task(task, (int)ni);
          allocated = true;
          break;
        }
        if (!allocated) backfill_fit_errors[job.uid][task->uid] = fe;
      }
    }
  }
};

// ---------------------------------------------------------------------------
// JSON entry points
// ---------------------------------------------------------------------------
static Value vstr(const std::string& s) { Value v; v.kind = Value::Str; v.s = s; return v; }
static Value vint(int64_t i) { Value v; v.kind = Value::Int; v.i = i; return v; }
static Value vdbl(double d) { Value v; v.kind = Value::Dbl; v.d = d; return v; }
static Value vbool(bool b) { Value v; v.kind = Value::Bool; v.b = b; return v; }
static Value vobj() { Value v; v.kind = Value::Obj; return v; }
static Value varr() { Value v; v.kind = Value::Arr; return v; }

static void write(std::string& out, const Value& v) {
  switch (v.kind) {
    case Value::Null: out += "null"; break;
    case Value::Bool: out += v.b ? "true" : "false"; break;
    case Value::Int: out += std::to_string(v.i); break;
    case Value::Dbl: {
      char buf[64];
      if (std::isfinite(v.d) && v.d == std::floor(v.d) && std::fabs(v.d) < 9e15) snprintf(buf, sizeof buf, "%.1f", v.d);
      else snprintf(buf, sizeof buf, "%.17g", v.d);
      out += buf;
      break;
    }
    case Value::Str: oj::esc(out, v.s); break;
    case Value::Arr:
      out += '[';
      for (size_t i = 0; i < v.a.size(); ++i) { if (i) out += ','; write(out, v.a[i]); }
      out += ']';
      break;
    case Value::Obj:
      out += '{';
      for (size_t i = 0; i < v.o.size(); ++i) {
        if (i) out += ',';
        oj::esc(out, v.o[i].first);
        out += ':';
        write(out, v.o[i].second);
      }
      out += '}';
      break;
  }
}

static Options parse_opts(const Value& in) {
  Options o;
  if (const Value* op = in.get("options")) {
    o.workers = (int)op->int_at("workers", 1);
    o.literal_affinity = op->bool_at("literal_affinity");
    o.max_tasks = op->int_at("max_tasks", -1);
  }
  return o;
}

static Value run_allocate(const Value& in) {
  Session s;
  s.opt = parse_opts(in);
  s.load(in);
  s.allocate();
  const bool backfill = in.str_at("op") == "allocate_backfill";  // the default action list (util.go:32)
  if (backfill) s.backfill();
  Value out = vobj();
  Value ev = varr();
  for (auto& e : s.events) {
    Value x = vobj();
    x.o.emplace_back("task", vstr(e.task_uid));
    x.o.emplace_back("node", vstr(e.node));
    x.o.emplace_back("kind", vstr(e.kind == Allocated ? "allocate" : "pipeline"));
    ev.a.push_back(x);
  }
  out.o.emplace_back("events", ev);
  Value b = vobj();
  for (auto& kv : s.binds) b.o.emplace_back(kv.first, vstr(kv.second));
  out.o.emplace_back("binds", b);
  Value fe = vobj();
  for (auto& jkv : s.jobs) {
    if (jkv.second.fit_errors.empty()) continue;
    Value j = vobj();
    for (auto& tkv : jkv.second.fit_errors) {
      Value h = vobj();
      for (auto& r : tkv.second.hist) h.o.emplace_back(r.first, vint(r.second));
      j.o.emplace_back(tkv.first, h);
    }
    fe.o.emplace_back(jkv.first, j);
  }
  out.o.emplace_back("fit_errors", fe);
  if (backfill) {
    Value bfe = vobj();
    for (auto& jkv : s.backfill_fit_errors) {
      Value j = vobj();
      for (auto& tkv : jkv.second) {
        Value h = vobj();
        for (auto& r : tkv.second.hist) h.o.emplace_back(r.first, vint(r.second));
        j.o.emplace_back(tkv.first, h);
      }
      bfe.o.emplace_back(jkv.first, j);
    }
    out.o.emplace_back("backfill_fit_errors", bfe);
  }
  Value st = vobj();
  for (auto& t : s.tasks) st.o.emplace_back(t.uid, vstr(status_name(t.status)));
  out.o.emplace_back("status", st);
  Value nodes = varr();
  for (auto& n : s.nodes) nodes.a.push_back(vstr(n.name));
  out.o.emplace_back("nodes", nodes);
  out.o.emplace_back("attempts", vint(s.attempts));
  out.o.emplace_back("elapsed_ms", vdbl(s.elapsed_ms));
  out.o.emplace_back("error", vstr(s.error));
  return out;
}

// Per-(task, node) mask and score at session-open state, for every node.
static Value run_eval(const Value& in) {
  Session s;
  s.opt = parse_opts(in);
  s.load(in);
  std::vector<const Task*> ts;
  std::map<std::string, const Task*> by_uid;
  for (auto& t : s.tasks) by_uid[t.uid] = &t;
  for (auto& u : in.arr_at("eval_tasks")) ts.push_back(by_uid.at(u.as_str()));
  Value out = vobj();
  Value nodes = varr();
  for (auto& n : s.nodes) nodes.a.push_back(vstr(n.name));
  out.o.emplace_back("nodes", nodes);
  Value res = varr();
  bool no = s.nodeorder_enabled();
  for (const Task* t : ts) {
    Value tr = vobj();
    Value reasons = varr(), scores = varr(), maperr = varr();
    std::vector<double> ipa;
    bool ipa_ok = no ? s.ipa_scores(t, &ipa) : true;
    for (size_t n = 0; n < s.nodes.size(); ++n) {
      PredResult p = s.alloc_predicate(t, (int)n);
      Value r = varr();
      for (auto& x : p.reasons) r.a.push_back(vstr(x));
      reasons.a.push_back(r);
      double sc = 0.0;
      bool ok = true;
      if (no) {
        double v;
        ok = s.node_order_fn(t, (int)n, &v);
        if (ok) sc = sc + v;
        if (ipa_ok) sc = sc + ipa[n] * (double)s.w_pa;
      }
      scores.a.push_back(vint((int64_t)sc));
      maperr.a.push_back(vbool(!ok));
    }
    tr.o.emplace_back("task", vstr(t->uid));
    tr.o.emplace_back("reasons", reasons);
    tr.o.emplace_back("score", scores);
    tr.o.emplace_back("map_error", maperr);
    tr.o.emplace_back("batch_error", vbool(!ipa_ok));
    res.a.push_back(tr);
  }
  out.o.emplace_back("tasks", res);
  return out;
}

// SortNodes order of preempt's sweep for each task of eval_tasks at session-open state.
static Value run_sort_nodes(const Value& in) {
  Session s;
  s.opt = parse_opts(in);
  s.load(in);
  std::map<std::string, const Task*> by_uid;
  for (auto& t : s.tasks) by_uid[t.uid] = &t;
  Value out = vobj(), res = varr();
  for (auto& u : in.arr_at("eval_tasks")) {
    Value tr = vobj(), order = varr(), scores = varr(), feas = varr(), hist = vobj();
    Session::Sweep sw;
    for (auto& p : s.sort_nodes(by_uid.at(u.as_str()), &sw)) {
      order.a.push_back(vstr(s.nodes[p.first].name));
      scores.a.push_back(vint((int64_t)p.second));
    }
    // util.PredicateNodes(task, nodes, ssn.PredicateFn): the feasible set in node order + the FitErrors
    std::map<std::string, int> h;
    for (size_t i = 0; i < sw.pred.size(); ++i) {
      if (sw.pred[i].ok) feas.a.push_back(vstr(s.nodes[i].name));
      else
        for (auto& r : sw.pred[i].reasons) h[r]++;
    }
    for (auto& kv : h) hist.o.emplace_back(kv.first, vint(kv.second));
    tr.o.emplace_back("feasible", feas);
    tr.o.emplace_back("fit_errors", hist);
    tr.o.emplace_back("task", vstr(u.as_str()));
    tr.o.emplace_back("order", order);
    tr.o.emplace_back("score", scores);
    res.a.push_back(tr);
  }
  out.o.emplace_back("tasks", res);
  return out;
}

// Resource / NodeInfo / pod-request primitives for the restated api unit tests.
static Value run_resource_op(const Value& in) {
  std::string op = in.str_at("op");
  Value out = vobj();
  auto R = [&](const char* k) { return Resource::from_json(*in.get(k)); };
  if (op == "LessEqual") out.o.emplace_back("result", vbool(R("l").less_equal(R("r"))));
  else if (op == "Less") out.o.emplace_back("result", vbool(R("l").less(R("r"))));
  else if (op == "IsEmpty") out.o.emplace_back("result", vbool(R("l").is_empty()));
  else if (op == "IsZero") out.o.emplace_back("result", vbool(R("l").is_zero(in.str_at("name"))));
  else if (op == "Add") { Resource l = R("l"); l.add(R("r")); out.o.emplace_back("result", l.to_json()); }
  else if (op == "Sub") { Resource l = R("l"); l.sub(R("r")); out.o.emplace_back("result", l.to_json()); }
  else if (op == "SetMaxResource") { Resource l = R("l"); l.set_max(R("r")); out.o.emplace_back("result", l.to_json()); }
  else if (op == "FitDelta") { Resource l = R("l"); l.fit_delta(R("r")); out.o.emplace_back("result", l.to_json()); }
  else if (op == "AddScalar") {
    Resource l = R("l");
    l.add_scalar(in.str_at("name"), in.get("quantity")->as_dbl());
    out.o.emplace_back("result", l.to_json());
  } else if (op == "NewResource") out.o.emplace_back("result", Resource::from_list(*in.get("list")).to_json());
  else if (op == "PodRequest") {
    Pod p = parse_pod(*in.get("pod"));
    out.o.emplace_back("resreq", pod_resreq(p).to_json());
    out.o.emplace_back("initreq", pod_initreq(p).to_json());
  } else if (op == "NodeTasks") {
    // NewNodeInfo + AddTask / RemoveTask (api/node_info.go:59-221)
    NodeSpec ns = parse_node(*in.get("node"));
    NodeI ni;
    ni.name = ns.name;
    ni.node = &ns;
    ni.idle = Resource::from_list(ns.alloc);
    ni.alloc = Resource::from_list(ns.alloc);
    ni.cap = Resource::from_list(ns.cap);
    std::deque<Pod> ps;
    std::deque<Task> tk;
    for (auto& pv : in.arr_at("pods")) {
      ps.push_back(parse_pod(pv));
      tk.emplace_back();
      Task& t = tk.back();
      t.pod = &ps.back();
      t.uid = ps.back().uid;
      t.status = get_task_status(ps.back());
      t.resreq = pod_resreq(ps.back());
      ni.add_task(&t);
    }
    for (auto& pv : in.arr_at("remove")) {
      Pod p = parse_pod(pv);
      for (size_t i = 0; i < ni.tasks.size(); ++i) {
        const Task* t = ni.tasks[i];
        if (t->pod->ns == p.ns && t->pod->name == p.name) {
          switch (t->status) {
            case Releasing: ni.releasing.sub(t->resreq); ni.idle.add(t->resreq); break;
            case Pipelined: ni.releasing.add(t->resreq); break;
            default: ni.idle.add(t->resreq);
          }
          ni.used.sub(t->resreq);
          ni.task_keys.erase(p.ns + "/" + p.name);
          ni.tasks.erase(ni.tasks.begin() + i);
          break;
        }
      }
    }
    out.o.emplace_back("idle", ni.idle.to_json());
    out.o.emplace_back("used", ni.used.to_json());
    out.o.emplace_back("releasing", ni.releasing.to_json());
    Value keys = varr();
    for (auto& k : ni.task_keys) keys.a.push_back(vstr(k));
    out.o.emplace_back("tasks", keys);
  } else if (op == "JobTasks") {
    // NewJobInfo + AddTaskInfo / DeleteTaskInfo (api/job_info.go:160-179, 239-283): Allocated,
    // TotalRequest and the TaskStatusIndex
    Job job;
    std::deque<Pod> ps;
    std::deque<Task> tk;
    auto mk = [&](const Value& pv) {
      ps.push_back(parse_pod(pv));
      tk.emplace_back();
      Task& t = tk.back();
      t.pod = &ps.back();
      t.uid = ps.back().uid;
      t.status = get_task_status(ps.back());
      t.resreq = pod_resreq(ps.back());
      t.initreq = pod_initreq(ps.back());
      return &t;
    };
    for (auto& pv : in.arr_at("pods")) job.add_task_info(mk(pv));
    for (auto& pv : in.arr_at("remove")) job.delete_task_info(mk(pv));
    out.o.emplace_back("allocated", job.allocated.to_json());
    out.o.emplace_back("total_request", job.total_request.to_json());
    Value idx = vobj();
    for (auto& kv : job.tsi) {
      Value u = varr();
      for (auto& tkv : kv.second) u.a.push_back(vstr(tkv.first));
      idx.o.emplace_back(status_name(kv.first), u);
    }
    out.o.emplace_back("status_index", idx);
    Value all = varr();
    for (auto& kv : job.tasks) all.a.push_back(vstr(kv.first));
    out.o.emplace_back("tasks", all);
  } else if (op == "IsScalarResourceName") {
    out.o.emplace_back("result", vbool(is_scalar_resource_name(in.str_at("name"))));
  } else if (op == "SelectorMatches") {
    // NodeSelectorRequirementsAsSelector(exprs).Matches(labels)
    Selector s;
    bool ok = node_reqs_as_selector(parse_reqs(*in.get("exprs")), &s);
    out.o.emplace_back("valid", vbool(ok));
    out.o.emplace_back("result", vbool(ok && s.matches(parse_labels(in.get("labels")))));
  } else {
    throw std::runtime_error("unknown op " + op);
  }
  return out;
}

}  // namespace oracle

extern "C" {
// oracle_call(json) -> malloc'd JSON string; free with oracle_free.
char* oracle_call(const char* json_in) {
  std::string out;
  try {
    oj::Value in = oj::parse(json_in);
    std::string op = in.str_at("op");
    oj::Value res;
    if (op == "allocate" || op == "allocate_backfill") res = oracle::run_allocate(in);
    else if (op == "eval") res = oracle::run_eval(in);
    else if (op == "sort_nodes") res = oracle::run_sort_nodes(in);
    else res = oracle::run_resource_op(in);
    oracle::write(out, res);
  } catch (const oracle::Panic& e) {
    out = std::string("{\"panic\":");
    oj::esc(out, e.what());
    out += "}";
  } catch (const std::exception& e) {
    out = std::string("{\"exception\":");
    oj::esc(out, e.what());
    out += "}";
  }
  char* r = (char*)malloc(out.size() + 1);
  memcpy(r, out.c_str(), out.size() + 1);
  return r;
}
void oracle_free(char* p) { free(p); }
}
