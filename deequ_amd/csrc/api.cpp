// api.cpp -- host runtime behind the C ABI (include/deequ_amd.h): expression decoding, the planner
// that maps a suite's aggregation functions onto fused column tasks, the device state, the
// Spark-partial-aggregate merge, and (de)serialisation for multi-GPU collectives.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <memory>
#include <string>
#include <tuple>
#include <vector>

#include "decimal.h"
#include "engine.h"
#include "kernels.h"
#include "jfmt.h"

using namespace dq;

// Every host wait on device work this file makes (stream / event synchronisations) is counted:
// dq_host_wait_count() lets tests assert how many a path takes (the state exchange: one, the
// read-back of the merged state).
#include <atomic>
static std::atomic<long long> g_host_waits{0};
static hipError_t host_wait(hipStream_t st) {
  g_host_waits.fetch_add(1, std::memory_order_relaxed);
  return hipStreamSynchronize(st);
}
static hipError_t host_wait_event(hipEvent_t ev) {
  g_host_waits.fetch_add(1, std::memory_order_relaxed);
  return hipEventSynchronize(ev);
}
extern "C" int64_t dq_host_wait_count(void) { return g_host_waits.load(std::memory_order_relaxed); }

// ------------------------------------------------------------------------------------------------
// Errors
// ------------------------------------------------------------------------------------------------
static thread_local std::string g_last_error;

dq_status dq::fail(dq_status code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}


extern "C" const char* dq_last_error(void) { return g_last_error.c_str(); }
extern "C" int dq_version(void) { return 100; }
extern "C" int dq_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

static bool is_numeric(int t) { return t >= DQ_INT8 && t <= DQ_FLOAT64; }
static bool is_integral(int t) { return t >= DQ_INT8 && t <= DQ_INT64; }
static bool is_floating(int t) { return t == DQ_FLOAT32 || t == DQ_FLOAT64; }
static bool is_decimal(int t) { return DQ_TYPE_ID(t) == DQ_DECIMAL128; }
// date / timestamp / decimal: types with no native arithmetic in the scan bodies' numeric paths
static bool is_temporal(int t) { return t == DQ_DATE32 || t == DQ_TIMESTAMP_US; }
// A well-formed type word (decimal: 1 <= p <= 38, 0 <= s <= p, nothing above bit 23).
static bool valid_type(int t) {
  if (is_decimal(t)) {
    const int p = DQ_DECIMAL_PRECISION(t), sc = DQ_DECIMAL_SCALE(t);
    return (t >> 24) == 0 && p >= 1 && p <= 38 && sc <= p;
  }
  return t >= DQ_BOOL && t <= DQ_TIMESTAMP_US;
}
// The physical layout a kernel that only compares / hashes values may treat a column as: a date is
// an int32 (hashInt, XxHash64Function on DateType), a timestamp an int64 (hashLong).
static int phys_type(int t) {
  if (t == DQ_DATE32) return DQ_INT32;
  if (t == DQ_TIMESTAMP_US) return DQ_INT64;
  return t;
}
static int type_size(int t) {
  if (is_decimal(t)) return 16;
  switch (t) {
    case DQ_DATE32: return 4;
    case DQ_TIMESTAMP_US: return 8;
    case DQ_INT8: return 1;
    case DQ_INT16: return 2;
    case DQ_INT32: return 4;
    case DQ_INT64: return 8;
    case DQ_FLOAT32: return 4;
    case DQ_FLOAT64: return 8;
    case DQ_UTF8: return 4;
    default: return 0;
  }
}

// ------------------------------------------------------------------------------------------------
// Expression trees
// ------------------------------------------------------------------------------------------------
struct Node {
  int op = 0;
  int col = -1;
  int64_t i = 0;
  double d = 0.0;
  std::string s;
  std::vector<std::unique_ptr<Node>> kids;
};

static bool parse_node(const int64_t* w, int n, int& pos, std::unique_ptr<Node>& out, int ncols,
                       int depth) {
  if (pos >= n || depth > 64) return false;
  auto node = std::make_unique<Node>();
  node->op = (int)w[pos++];
  auto child = [&](void) -> bool {
    std::unique_ptr<Node> c;
    if (!parse_node(w, n, pos, c, ncols, depth + 1)) return false;
    node->kids.push_back(std::move(c));
    return true;
  };
  switch (node->op) {
    case DQ_X_COL:
      if (pos >= n) return false;
      node->col = (int)w[pos++];
      if (node->col < 0 || node->col >= ncols) return false;
      break;
    case DQ_X_NULL: break;
    case DQ_X_BOOL:
    case DQ_X_I64:
      if (pos >= n) return false;
      node->i = w[pos++];
      break;
    case DQ_X_F64:
      if (pos >= n) return false;
      memcpy(&node->d, &w[pos++], 8);
      break;
    case DQ_X_DEC128:  // i = low word, d = high word's bits
      if (pos + 1 >= n) return false;
      node->i = w[pos++];
      memcpy(&node->d, &w[pos++], 8);
      break;
    case DQ_X_STR: {
      if (pos >= n) return false;
      int64_t nb = w[pos++];
      int64_t nw = (nb + 7) / 8;
      if (nb < 0 || pos + nw > n) return false;
      node->s.assign(reinterpret_cast<const char*>(&w[pos]), (size_t)nb);
      pos += (int)nw;
      break;
    }
    case DQ_X_IS_NULL:
    case DQ_X_IS_NOT_NULL:
    case DQ_X_NOT:
    case DQ_X_CAST_F64:
    case DQ_X_CAST_F32:
      if (!child()) return false;
      break;
    case DQ_X_AND:
    case DQ_X_OR:
    case DQ_X_EQ:
    case DQ_X_NE:
    case DQ_X_LT:
    case DQ_X_LE:
    case DQ_X_GT:
    case DQ_X_GE:
    case DQ_X_EQ_NULL_SAFE:
      if (!child() || !child()) return false;
      break;
    case DQ_X_REGEX: {
      if (pos + 1 >= n) return false;
      node->i = w[pos++];  // null_mode
      const int64_t nb = w[pos++];
      const int64_t nw = (nb + 7) / 8;
      if (nb < 16 + 256 || pos + nw > n) return false;
      node->s.assign(reinterpret_cast<const char*>(&w[pos]), (size_t)nb);
      pos += (int)nw;
      // validate the automaton's shape before any device code indexes it
      int32_t hd[4];
      memcpy(hd, node->s.data(), 16);
      const int64_t ns = hd[0], nc = hd[1], st = hd[2];
      if (ns < 1 || ns > 65535 || nc < 2 || nc > 257 || st < 0 || st >= ns) return false;
      const int64_t need = 16 + 256 + ((ns + 3) & ~3LL) + 2 * ns * nc;
      if (nb != need) return false;
      const uint8_t* cls = reinterpret_cast<const uint8_t*>(node->s.data()) + 16;
      for (int b = 0; b < 256; ++b)
        if (cls[b] >= nc - 1) return false;
      const uint16_t* nx = reinterpret_cast<const uint16_t*>(node->s.data() + 16 + 256 + ((ns + 3) & ~3LL));
      for (int64_t k = 0; k < ns * nc; ++k) {
        uint16_t v;
        memcpy(&v, nx + k, 2);
        if (v >= ns) return false;
      }
      if (!child()) return false;
      break;
    }
    case DQ_X_IN: {
      if (pos >= n) return false;
      int64_t items = w[pos++];
      if (items < 0 || items > 4096) return false;
      for (int64_t k = 0; k < items + 1; ++k)
        if (!child()) return false;
      break;
    }
    default: return false;
  }
  out = std::move(node);
  return true;
}

static bool is_cmp(int op) { return op >= DQ_X_EQ && op <= DQ_X_GE; }
static int flip_cmp(int op) {
  switch (op) {
    case DQ_X_LT: return DQ_X_GT;
    case DQ_X_LE: return DQ_X_GE;
    case DQ_X_GT: return DQ_X_LT;
    case DQ_X_GE: return DQ_X_LE;
    default: return op;
  }
}

static void compile_postfix(const Node& n, std::vector<XInstr>& prog, std::string& pool) {
  for (auto& k : n.kids) compile_postfix(*k, prog, pool);
  XInstr ins{0, 0, 0};
  switch (n.op) {
    case DQ_X_COL: ins = {XI_COL, n.col, 0}; break;
    case DQ_X_NULL: ins = {XI_NULL, 0, 0}; break;
    case DQ_X_BOOL: ins = {XI_BOOL, 0, n.i ? 1 : 0}; break;
    case DQ_X_I64: ins = {XI_I64, 0, n.i}; break;
    case DQ_X_F64: {
      int64_t b;
      memcpy(&b, &n.d, 8);
      ins = {XI_F64, 0, b};
      break;
    }
    case DQ_X_DEC128: {  // two words: the low word's instruction, then the high word's
      int64_t hi;
      memcpy(&hi, &n.d, 8);
      prog.push_back(XInstr{XI_DEC128, 0, n.i});
      ins = {XI_DEC128_HI, 0, hi};
      break;
    }
    case DQ_X_STR: {
      while (pool.size() % 4) pool.push_back('\0');
      ins = {XI_STR, (int32_t)n.s.size(), (int64_t)pool.size()};
      pool += n.s;
      break;
    }
    case DQ_X_IS_NULL: ins = {XI_IS_NULL, 0, 0}; break;
    case DQ_X_IS_NOT_NULL: ins = {XI_IS_NOT_NULL, 0, 0}; break;
    case DQ_X_NOT: ins = {XI_NOT, 0, 0}; break;
    case DQ_X_AND: ins = {XI_AND, 0, 0}; break;
    case DQ_X_OR: ins = {XI_OR, 0, 0}; break;
    case DQ_X_IN: ins = {XI_IN, (int32_t)n.kids.size() - 1, 0}; break;
    case DQ_X_CAST_F64: ins = {XI_CAST_F64, 0, 0}; break;
    case DQ_X_CAST_F32: ins = {XI_CAST_F64, 1, 0}; break;  // a = 1: round to float
    case DQ_X_REGEX: {
      while (pool.size() % 8) pool.push_back('\0');
      ins = {XI_REGEX, (int32_t)n.i, (int64_t)pool.size()};
      pool += n.s;
      break;
    }
    default: ins = {XI_CMP, n.op, 0}; break;
  }
  prog.push_back(ins);
}

// CAST(x AS FLOAT) of a string operand (a utf8 column or a string literal): Spark parses it with
// Float.parseFloat, which the interpreter does not restate (it would parse a double and skip the
// float rounding), so the plan refuses it rather than compute a different value.
static bool casts_string_to_float(const Node& n, const std::vector<int32_t>& types) {
  if (n.op == DQ_X_CAST_F32 && !n.kids.empty()) {
    const Node& x = *n.kids[0];
    if (x.op == DQ_X_STR || (x.op == DQ_X_COL && types[x.col] == DQ_UTF8)) return true;
  }
  for (auto& k : n.kids)
    if (casts_string_to_float(*k, types)) return true;
  return false;
}

// Where a decimal / date / timestamp column may appear in an expression (deequ_amd.h, DQ_X_DEC128):
// the interpreter has no other arithmetic for them, so anything else is refused, never evaluated
// in the wrong domain.  Returns false and names the offending use in `why`.
static bool typed_uses_ok(const Node& n, const std::vector<int32_t>& types, std::string& why) {
  auto dec_col = [&](const Node* x) { return x->op == DQ_X_COL && is_decimal(types[x->col]); };
  auto special = [&](const Node* x) {
    return x->op == DQ_X_COL && (is_decimal(types[x->col]) || is_temporal(types[x->col]));
  };
  switch (n.op) {
    case DQ_X_COL:
      if (special(&n)) {
        why = "a decimal / date / timestamp column used outside IS [NOT] NULL, a comparison with a "
              "decimal literal, CAST AS DOUBLE or a regex";
        return false;
      }
      return true;
    case DQ_X_DEC128:
      why = "a decimal literal outside a comparison with a decimal column";
      return false;
    case DQ_X_IS_NULL:
    case DQ_X_IS_NOT_NULL:
    case DQ_X_REGEX:
      if (special(n.kids[0].get())) return true;
      break;
    case DQ_X_CAST_F64:
      if (dec_col(n.kids[0].get())) return true;
      break;
    case DQ_X_IN:
      if (dec_col(n.kids[0].get())) {
        for (size_t k = 1; k < n.kids.size(); ++k)
          if (n.kids[k]->op != DQ_X_DEC128 && n.kids[k]->op != DQ_X_NULL) {
            why = "a decimal column IN a list of non-decimal items";
            return false;
          }
        return true;
      }
      break;
    default:
      if (is_cmp(n.op) || n.op == DQ_X_EQ_NULL_SAFE) {
        const Node* a = n.kids[0].get();
        const Node* b = n.kids[1].get();
        if (dec_col(a) && (b->op == DQ_X_DEC128 || b->op == DQ_X_NULL)) return true;
        if (dec_col(b) && (a->op == DQ_X_DEC128 || a->op == DQ_X_NULL)) return true;
      }
      break;
  }
  for (auto& k : n.kids)
    if (!typed_uses_ok(*k, types, why)) return false;
  return true;
}

static int stack_depth(const Node& n) {
  int best = 0, k = 0;
  for (auto& c : n.kids) best = std::max(best, k++ + stack_depth(*c));
  return std::max(best, 1);
}

// ------------------------------------------------------------------------------------------------
// Predicate fusion: recognise the forms Check emits so they run inside a column task.
// ------------------------------------------------------------------------------------------------
struct CmpLeaf {
  int col = -1;
  int op = 0;
  bool lit_f64 = false;
  int64_t li = 0;
  double ld = 0.0;
};

static bool leaf_cmp(const Node& n, const std::vector<int32_t>& types, CmpLeaf& out) {
  if (!is_cmp(n.op)) return false;
  const Node* a = n.kids[0].get();
  const Node* b = n.kids[1].get();
  int op = n.op;
  auto is_lit = [](const Node* x) { return x->op == DQ_X_I64 || x->op == DQ_X_F64; };
  auto colref = [&](const Node* x) -> int {
    if (x->op == DQ_X_COL && is_numeric(types[x->col])) return x->col;
    return -1;
  };
  if (colref(b) >= 0 && is_lit(a)) {
    std::swap(a, b);
    op = flip_cmp(op);
  }
  int c = colref(a);
  if (c < 0 || !is_lit(b)) return false;
  out.col = c;
  out.op = op;
  out.lit_f64 = b->op == DQ_X_F64;
  out.li = b->i;
  out.ld = b->op == DQ_X_F64 ? b->d : (double)b->i;
  return true;
}

// [col IS NULL OR] (cmp [AND cmp])  on one numeric column
static bool fuse_numeric(const Node& n, const std::vector<int32_t>& types, int& col, NumPred& p) {
  p = NumPred{};
  const Node* body = &n;
  int null_col = -1;
  if (n.op == DQ_X_OR && n.kids[0]->op == DQ_X_IS_NULL && n.kids[0]->kids[0]->op == DQ_X_COL) {
    null_col = n.kids[0]->kids[0]->col;
    body = n.kids[1].get();
  }
  CmpLeaf a, b;
  bool two = false;
  if (body->op == DQ_X_AND) {
    if (!leaf_cmp(*body->kids[0], types, a) || !leaf_cmp(*body->kids[1], types, b)) return false;
    if (a.col != b.col) return false;
    two = true;
  } else if (!leaf_cmp(*body, types, a)) {
    return false;
  }
  if (null_col >= 0 && null_col != a.col) return false;
  const bool fcol = is_floating(types[a.col]);
  const bool as_double = fcol || a.lit_f64 || (two && b.lit_f64);
  // both comparisons must live in the same domain as Spark evaluates them
  if (two && !fcol && (a.lit_f64 != b.lit_f64)) return false;
  if (as_double && !fcol && types[a.col] == DQ_INT64) {
    // Spark casts the long column to double for a double literal: same here (exact below 2^53)
  }
  col = a.col;
  p.op1 = a.op;
  p.op2 = two ? b.op : 0;
  p.as_double = as_double ? 1 : 0;
  p.null_is_true = null_col >= 0 ? 1 : 0;
  p.lo_i = a.li;
  p.lo_d = a.ld;
  p.hi_i = two ? b.li : 0;
  p.hi_d = two ? b.ld : 0.0;
  return true;
}

struct StrIn {
  int col = -1;
  bool negate = false;
  bool null_is_true = false;
  std::vector<std::string> list;
};

static bool fuse_str_in_body(const Node& n, const std::vector<int32_t>& types, StrIn& s) {
  if (n.op == DQ_X_NOT) {
    if (!fuse_str_in_body(*n.kids[0], types, s)) return false;
    s.negate = !s.negate;
    return true;
  }
  if (n.op == DQ_X_IN) {
    const Node& x = *n.kids[0];
    if (x.op != DQ_X_COL || types[x.col] != DQ_UTF8) return false;
    for (size_t k = 1; k < n.kids.size(); ++k) {
      if (n.kids[k]->op != DQ_X_STR) return false;
      s.list.push_back(n.kids[k]->s);
    }
    s.col = x.col;
    return true;
  }
  if (n.op == DQ_X_EQ || n.op == DQ_X_NE) {
    const Node* a = n.kids[0].get();
    const Node* b = n.kids[1].get();
    if (a->op == DQ_X_STR) std::swap(a, b);
    if (a->op != DQ_X_COL || types[a->col] != DQ_UTF8 || b->op != DQ_X_STR) return false;
    s.col = a->col;
    s.list.push_back(b->s);
    s.negate = n.op == DQ_X_NE;
    return true;
  }
  return false;
}

static bool fuse_str_in(const Node& n, const std::vector<int32_t>& types, StrIn& s) {
  s = StrIn{};
  if (n.op == DQ_X_OR && n.kids[0]->op == DQ_X_IS_NULL && n.kids[0]->kids[0]->op == DQ_X_COL) {
    int nc = n.kids[0]->kids[0]->col;
    if (!fuse_str_in_body(*n.kids[1], types, s)) return false;
    if (s.col != nc) return false;
    s.null_is_true = true;
    return true;
  }
  return fuse_str_in_body(n, types, s);
}

// ------------------------------------------------------------------------------------------------
// Plan
// ------------------------------------------------------------------------------------------------
enum SlotSrc { SRC_ROWS = 1, SRC_TASK = 2 };

struct Slot {
  int kind = 0;    // dq_agg_kind
  int src = 0;     // SlotSrc
  int task = -1;   // task index
  int field = 0;   // pred index for fused numeric predicates, else 0
  int col_type = 0;
  bool fused_pred = false;
  bool notnull_rows = false;  // COUNT_NOTNULL: NULL only when no rows
};

struct TaskPlan {
  int kind = 0;
  int col = -1, col2 = -1;
  int where = -1;      // materialised where expression index (into plan->mat)
  int bool_expr = -1;  // TK_BOOLMAP counted expression (into plan->mat)
  int n_preds = 0;
  NumPred preds[kMaxPreds];
  StrIn str;
  int out = 0;
  int hll_out = -1;
  // TK_COMOMENTS fused with an ApproxCountDistinct of one of its columns (BC_CORR_HLL): the HLL
  // task's register file and which column it hashes (0 = col, 1 = col2)
  int fused_hll = -1, hll_side = 0;
  bool carried = false;  // TK_HLL whose rows a fused co-moment task hashes: no items of its own
};

struct MatExpr {
  int expr = -1;                // index in desc exprs
  std::vector<XInstr> prog;
  std::string pool;
};

struct dq_plan {
  std::vector<int32_t> types;
  std::vector<std::unique_ptr<Node>> exprs;
  std::vector<dq_agg> aggs;
  std::vector<Slot> slots;
  std::vector<TaskPlan> tasks;
  std::vector<MatExpr> mat;     // materialised expressions (where filters + unfusable predicates)
  std::map<int, int> mat_of;    // expr index -> mat index
  int n_hll = 0;
  bool full = false;            // needs the full kernel family (hashing / co-moments / int8/16)
};

// Scan kernel instantiation that runs a task (kernels.h BodyClass).
static int body_class(const dq_plan* p, const TaskPlan& t) {
  switch (t.kind) {
    case TK_NUMERIC:
      switch (p->types[t.col]) {
        case DQ_INT8: return BC_NUM_I8;
        case DQ_INT16: return BC_NUM_I16;
        case DQ_INT32: return BC_NUM_I32;
        case DQ_INT64: return BC_NUM_I64;
        case DQ_FLOAT32: return BC_NUM_F32;
        default: return BC_NUM_F64;
      }
    case TK_VALIDITY:
    case TK_BOOLMAP: return BC_BITS;
    case TK_STR_IN: return BC_STR_IN;
    case TK_DTYPE: return BC_DTYPE;
    case TK_COMOMENTS: return t.fused_hll >= 0 ? BC_CORR_HLL : BC_CORR;
    case TK_DECIMAL: return BC_DECIMAL;
    default: return BC_HLL;
  }
}

static int mat_index(dq_plan* p, int expr) {
  auto it = p->mat_of.find(expr);
  if (it != p->mat_of.end()) return it->second;
  MatExpr m;
  m.expr = expr;
  compile_postfix(*p->exprs[expr], m.prog, m.pool);
  int idx = (int)p->mat.size();
  p->mat.push_back(std::move(m));
  p->mat_of[expr] = idx;
  return idx;
}

static int find_or_add_task(dq_plan* p, int kind, int col, int col2, int where) {
  for (size_t k = 0; k < p->tasks.size(); ++k) {
    const TaskPlan& t = p->tasks[k];
    if (t.kind == kind && t.col == col && t.col2 == col2 && t.where == where && kind != TK_STR_IN &&
        kind != TK_BOOLMAP)
      return (int)k;
  }
  TaskPlan t;
  t.kind = kind;
  t.col = col;
  t.col2 = col2;
  t.where = where;
  t.out = (int)p->tasks.size();
  if (kind == TK_HLL) t.hll_out = p->n_hll++;
  p->tasks.push_back(t);
  return (int)p->tasks.size() - 1;
}

extern "C" dq_status dq_plan_create(const dq_plan_desc* desc, dq_plan** out) {
  if (!desc || !out) return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  *out = nullptr;
  if (desc->n_columns < 0 || desc->n_exprs < 0 || desc->n_aggs < 0)
    return fail(DQ_ERR_INVALID_ARGUMENT, "negative counts in plan description");
  auto p = std::make_unique<dq_plan>();
  p->types.assign(desc->column_types, desc->column_types + desc->n_columns);
  for (int t : p->types)
    if (!valid_type(t)) return fail(DQ_ERR_INVALID_ARGUMENT, "unknown column type %d", t);
  for (int e = 0; e < desc->n_exprs; ++e) {
    std::unique_ptr<Node> n;
    int pos = 0;
    if (!parse_node(desc->exprs[e].words, desc->exprs[e].n_words, pos, n, desc->n_columns, 0) ||
        pos != desc->exprs[e].n_words)
      return fail(DQ_ERR_INVALID_ARGUMENT, "malformed expression %d", e);
    if (stack_depth(*n) > kMaxStack)
      return fail(DQ_ERR_UNSUPPORTED, "expression %d nests deeper than %d", e, kMaxStack);
    if (casts_string_to_float(*n, p->types))
      return fail(DQ_ERR_UNSUPPORTED, "expression %d casts a string to FLOAT", e);
    std::string why;
    if (!typed_uses_ok(*n, p->types, why)) return fail(DQ_ERR_UNSUPPORTED, "expression %d: %s", e, why.c_str());
    p->exprs.push_back(std::move(n));
  }
  p->aggs.assign(desc->aggs, desc->aggs + desc->n_aggs);

  auto check_col = [&](int c) -> dq_status {
    if (c < 0 || c >= desc->n_columns) return fail(DQ_ERR_NO_SUCH_COLUMN, "no such column %d", c);
    return DQ_OK;
  };
  auto where_of = [&](const dq_agg& a, int& w) -> dq_status {
    w = -1;
    if (a.where < 0) return DQ_OK;
    if (a.where >= desc->n_exprs) return fail(DQ_ERR_INVALID_ARGUMENT, "bad where index");
    w = mat_index(p.get(), a.where);
    return DQ_OK;
  };

  for (const dq_agg& a : p->aggs) {
    Slot s;
    s.kind = a.kind;
    int w = -1;
    dq_status st;
    switch (a.kind) {
      case DQ_AGG_COUNT_ALL: s.src = SRC_ROWS; break;
      case DQ_AGG_COUNT_NOTNULL: {
        if ((st = check_col(a.col)) != DQ_OK) return st;
        if ((st = where_of(a, w)) != DQ_OK) return st;
        s.src = SRC_TASK;
        s.notnull_rows = true;
        // share the numeric (decimal) task when one exists for (col, where); else a popcount task
        int found = -1;
        for (size_t k = 0; k < p->tasks.size(); ++k)
          if ((p->tasks[k].kind == TK_NUMERIC || p->tasks[k].kind == TK_DECIMAL) &&
              p->tasks[k].col == a.col && p->tasks[k].where == w)
            found = (int)k;
        s.task = found >= 0 ? found : find_or_add_task(p.get(), TK_VALIDITY, a.col, -1, w);
        break;
      }
      case DQ_AGG_COUNT_TRUE: {
        if (a.expr < 0 || a.expr >= desc->n_exprs)
          return fail(DQ_ERR_INVALID_ARGUMENT, "COUNT_TRUE needs an expression");
        if ((st = where_of(a, w)) != DQ_OK) return st;
        s.src = SRC_TASK;
        const Node& e = *p->exprs[a.expr];
        int col;
        NumPred np;
        StrIn si;
        // a where filter counted by itself (conditionalCount) reuses its bitmap
        if (p->mat_of.count(a.expr) && w < 0) {
          TaskPlan t;
          t.kind = TK_BOOLMAP;
          t.bool_expr = p->mat_of[a.expr];
          t.out = (int)p->tasks.size();
          p->tasks.push_back(t);
          s.task = t.out;
        } else if (fuse_numeric(e, p->types, col, np)) {
          int ti = find_or_add_task(p.get(), TK_NUMERIC, col, -1, w);
          TaskPlan& t = p->tasks[ti];
          if (t.n_preds < kMaxPreds) {
            t.preds[t.n_preds] = np;
            s.task = ti;
            s.field = t.n_preds++;
            s.fused_pred = true;
          } else {
            TaskPlan b;
            b.kind = TK_BOOLMAP;
            b.where = w;
            b.bool_expr = mat_index(p.get(), a.expr);
            b.out = (int)p->tasks.size();
            p->tasks.push_back(b);
            s.task = b.out;
          }
        } else if (fuse_str_in(e, p->types, si) && si.list.size() <= 256) {
          TaskPlan t;
          t.kind = TK_STR_IN;
          t.col = si.col;
          t.where = w;
          t.str = si;
          t.out = (int)p->tasks.size();
          p->tasks.push_back(t);
          s.task = t.out;
        } else {
          TaskPlan t;
          t.kind = TK_BOOLMAP;
          t.where = w;
          t.bool_expr = mat_index(p.get(), a.expr);
          t.out = (int)p->tasks.size();
          p->tasks.push_back(t);
          s.task = t.out;
        }
        break;
      }
      case DQ_AGG_SUM:
      case DQ_AGG_MIN:
      case DQ_AGG_MAX:
      case DQ_AGG_STDDEV_POP: {
        if ((st = check_col(a.col)) != DQ_OK) return st;
        if (!is_numeric(p->types[a.col]) && !is_decimal(p->types[a.col]))
          return fail(DQ_ERR_WRONG_TYPE, "column %d is not numeric", a.col);
        if ((st = where_of(a, w)) != DQ_OK) return st;
        s.src = SRC_TASK;
        s.task = find_or_add_task(p.get(), is_decimal(p->types[a.col]) ? TK_DECIMAL : TK_NUMERIC,
                                  a.col, -1, w);
        s.col_type = p->types[a.col];
        break;
      }
      case DQ_AGG_CORR: {
        if ((st = check_col(a.col)) != DQ_OK) return st;
        if ((st = check_col(a.col2)) != DQ_OK) return st;
        if (is_decimal(p->types[a.col]) || is_decimal(p->types[a.col2]))
          return fail(DQ_ERR_UNSUPPORTED, "correlation over a decimal column: cast it to double "
                                          "first (the engine's co-moment bodies read Long / Double)");
        if (!is_numeric(p->types[a.col]) || !is_numeric(p->types[a.col2]))
          return fail(DQ_ERR_WRONG_TYPE, "correlation needs numeric columns");
        if ((st = where_of(a, w)) != DQ_OK) return st;
        s.src = SRC_TASK;
        s.task = find_or_add_task(p.get(), TK_COMOMENTS, a.col, a.col2, w);
        break;
      }
      case DQ_AGG_HLL: {
        if ((st = check_col(a.col)) != DQ_OK) return st;
        if ((st = where_of(a, w)) != DQ_OK) return st;
        s.src = SRC_TASK;
        s.task = find_or_add_task(p.get(), TK_HLL, a.col, -1, w);
        break;
      }
      case DQ_AGG_DTYPE: {
        if ((st = check_col(a.col)) != DQ_OK) return st;
        if ((st = where_of(a, w)) != DQ_OK) return st;
        s.src = SRC_TASK;
        s.task = find_or_add_task(p.get(), TK_DTYPE, a.col, -1, w);
        break;
      }
      default: return fail(DQ_ERR_INVALID_ARGUMENT, "unknown aggregation kind %d", a.kind);
    }
    p->slots.push_back(s);
  }
  // COUNT_NOTNULL slots that picked a validity task before a numeric task for the same
  // (col, where) appeared are re-pointed so the column is read once.
  for (Slot& s : p->slots) {
    if (s.kind != DQ_AGG_COUNT_NOTNULL) continue;
    const TaskPlan& t = p->tasks[s.task];
    for (size_t k = 0; k < p->tasks.size(); ++k)
      if ((p->tasks[k].kind == TK_NUMERIC || p->tasks[k].kind == TK_DECIMAL) &&
          p->tasks[k].col == t.col && p->tasks[k].where == t.where)
        s.task = (int)k;
  }
  // drop validity tasks nobody references any more, renumber
  std::vector<int> used(p->tasks.size(), 0);
  for (const Slot& s : p->slots)
    if (s.task >= 0) used[s.task] = 1;
  std::vector<int> remap(p->tasks.size(), -1);
  std::vector<TaskPlan> kept;
  int n_hll = 0;
  for (size_t k = 0; k < p->tasks.size(); ++k) {
    if (!used[k]) continue;
    remap[k] = (int)kept.size();
    TaskPlan t = p->tasks[k];
    t.out = (int)kept.size();
    if (t.kind == TK_HLL) t.hll_out = n_hll++;
    kept.push_back(t);
  }
  p->tasks.swap(kept);
  p->n_hll = n_hll;
  for (Slot& s : p->slots)
    if (s.task >= 0) s.task = remap[s.task];
  for (const TaskPlan& t : p->tasks)
    if (t.kind == TK_HLL || t.kind == TK_COMOMENTS) p->full = true;
  // ApproxCountDistinct(c) beside Correlation(c, d) or (d, c) under the same where: one pass reads
  // both columns and feeds the co-moments and c's HLL registers (BC_CORR_HLL).  8-byte columns
  // only (the vector path both bodies share).  DQ_NO_FUSE=1 keeps two passes (A/B measurement).
  if (!getenv("DQ_NO_FUSE")) {
    auto wide = [&](int col) { return p->types[col] == DQ_INT64 || p->types[col] == DQ_FLOAT64; };
    for (TaskPlan& h : p->tasks) {
      if (h.kind != TK_HLL || !wide(h.col)) continue;
      for (TaskPlan& c : p->tasks) {
        if (c.kind != TK_COMOMENTS || c.fused_hll >= 0 || c.where != h.where) continue;
        if (!wide(c.col) || !wide(c.col2) || (c.col != h.col && c.col2 != h.col)) continue;
        c.fused_hll = h.hll_out;
        c.hll_side = c.col == h.col ? 0 : 1;
        h.carried = true;
        break;
      }
    }
  }
  // each workgroup keeps every HLL task's 512 registers in LDS (2 KiB per task)
  if (p->n_hll > 32)
    return fail(DQ_ERR_UNSUPPORTED, "%d ApproxCountDistinct aggregations in one plan (max 32)",
                p->n_hll);
  *out = p.release();
  return DQ_OK;
}

extern "C" void dq_plan_destroy(dq_plan* plan) { delete plan; }

static const char* kind_name(int k) {
  switch (k) {
    case TK_NUMERIC: return "numeric";
    case TK_VALIDITY: return "validity";
    case TK_STR_IN: return "str_in";
    case TK_BOOLMAP: return "boolmap";
    case TK_COMOMENTS: return "comoments";
    case TK_HLL: return "hll";
    case TK_DTYPE: return "dtype";
    case TK_DECIMAL: return "decimal";
    default: return "?";
  }
}

extern "C" dq_status dq_plan_explain(const dq_plan* plan, char* buf, size_t buf_len) {
  if (!plan || !buf || buf_len == 0) return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  std::string s;
  char line[256];
  for (size_t k = 0; k < plan->mat.size(); ++k) {
    snprintf(line, sizeof(line), "expr[%zu] = bitmap of expression %d (%zu instructions)\n", k,
             plan->mat[k].expr, plan->mat[k].prog.size());
    s += line;
  }
  for (const TaskPlan& t : plan->tasks) {
    char fused[64] = "";
    if (t.fused_hll >= 0) snprintf(fused, sizeof(fused), " +hll[%d] of col%s", t.fused_hll, t.hll_side ? "2" : "");
    if (t.carried) snprintf(fused, sizeof(fused), " (rows hashed by a fused co-moment pass)");
    snprintf(line, sizeof(line), "task[%d] %s col=%d col2=%d where=%d preds=%d list=%zu%s%s\n", t.out,
             kind_name(t.kind), t.col, t.col2, t.where, t.n_preds, t.str.list.size(),
             t.bool_expr >= 0 ? " (expr bitmap)" : "", fused);
    s += line;
  }
  snprintf(line, sizeof(line), "launches per batch: %d\n", dq_plan_launches_per_batch(plan));
  s += line;
  size_t n = std::min(buf_len - 1, s.size());
  memcpy(buf, s.data(), n);
  buf[n] = '\0';
  return DQ_OK;
}

extern "C" int dq_plan_launches_per_batch(const dq_plan* plan) {
  if (!plan) return 0;
  int classes = 0, hll = 0;
  for (int c = 0; c < kBodyClasses; ++c) {
    bool used = false;
    for (const TaskPlan& t : plan->tasks) used = used || (body_class(plan, t) == c && !t.carried);
    if (c == BC_HLL || c == BC_CORR_HLL || c == BC_DECIMAL) hll += used ? 1 : 0;  // own launches
    else classes += used ? 1 : 0;
  }
  // two or more body classes share one mixed launch (dq_scan_device_batches); HLL joins it when
  // its LDS registers fit (kMixedHllMax)
  bool hll_alone = false;  // an unfused HLL task (it may join the mixed launch)
  for (const TaskPlan& t : plan->tasks) hll_alone = hll_alone || (t.kind == TK_HLL && !t.carried);
  if (hll_alone && plan->n_hll <= kMixedHllMax && classes >= 1) {
    classes += 1;
    hll -= 1;
  }
  if (classes >= 2 && !getenv("DQ_NO_MIXED")) classes = 1;
  // expression bitmaps + the scan launches + the finalize launch
  return (int)plan->mat.size() + classes + hll + (plan->tasks.empty() ? 0 : 1);
}

// ------------------------------------------------------------------------------------------------
// State
// ------------------------------------------------------------------------------------------------
struct dq_state {
  const dq_plan* plan = nullptr;
  int device = 0;
  int grid[kQueues] = {};        // persistent grid of each scan kernel (+ the mixed kernel)
  int mix_hll = 0;               // HLL tasks carried by the mixed launch (0: HLL launches alone)
  hipStream_t stream = nullptr;
  bool stream_set = false;
  // host mirror
  std::vector<Acc> acc;
  std::vector<uint8_t> hll;
  int64_t rows = 0;
  bool host_dirty = false;   // host mirror newer than device (after merge / deserialize / reset)
  // reset since the last scan: the next scan's finalize starts from the initial values instead of
  // reading the device accumulators (dq_state_reset then queues no copies or memsets)
  bool reset_pending = false;
  bool synced = true;        // host mirror reflects every scanned batch
  // pinned staging of the host mirror: resets upload it and syncs read it back with async copies
  // on the state's stream and one stream synchronisation, instead of pageable hipMemcpy calls
  // that each block the host
  void* h_pin = nullptr;
  size_t h_pin_cap = 0;
  bool pin_pending = false;  // an async copy from h_pin may still be queued
  // device
  DevBuf<Acc> d_acc, d_partial, d_partial2;
  DevBuf<uint8_t> d_hll;
  DevBuf<uint32_t> d_hll_stage;  // per-launch HLL registers (u32), kept zero between launches
  DevBuf<uint32_t> d_fin_arrivals;  // finalize: per task, its workgroups done (kept zero)
  DevBuf<int64_t> d_rows;        // the merged row count of an exchange (dq_state_exchange_unpack)
  DevBuf<int32_t> d_kinds;       // the plan's task kinds (the exchange kernels), uploaded once
  std::vector<int32_t> h_kinds;  // (their source, alive while the upload may be queued)
  bool kinds_ready = false;
  hipEvent_t ev_xchg = nullptr;  // orders the exchange kernels and the collectives' stream
  bool rows_on_device = false;   // ... not yet read back (dq_state_sync reads it with the rest)
  DevBuf<uint32_t> d_queue;      // work-item counters of the scan kernels, kept zero between launches
  DevBuf<uint32_t> d_order[2];   // mixed launch: queue position -> item (per descriptor slot)
  std::vector<uint32_t> order_sig[2];  // the descriptors and launches d_order[slot] was built for
  std::vector<size_t> order_off[2], order_len[2];  // per queue group: its order list in d_order
  uint32_t* h_order[2] = {nullptr, nullptr};  // pinned staging of d_order[slot] (async upload)
  size_t h_order_cap[2] = {0, 0};
  DevBuf<TaskDesc> d_tasks[2];
  TaskDesc* h_tasks[2] = {nullptr, nullptr};
  size_t h_tasks_cap[2] = {0, 0};
  hipEvent_t ev[2] = {nullptr, nullptr};
  bool ev_used[2] = {false, false};
  int flip = 0;
  DevBuf<uint64_t> d_bitmaps;   // per materialised expression: value words then validity words
  size_t bitmap_words = 0;      // words per bitmap
  DevBuf<XInstr> d_prog;
  std::vector<int> prog_off;    // per mat expr: offset into d_prog
  DevBuf<uint8_t> d_pool;
  std::vector<int64_t> pool_off;
  // per mat expr: PatternMatch over a utf8 column runs regex_find_kernel on a fused table in
  // d_pool (col < 0: the interpreter)
  struct RegexRun {
    int col = -1, null_mode = 0, ns = 0, start = 0;
    int64_t table_off = 0;
  };
  std::vector<RegexRun> rx;
  DevBuf<DevCol> d_cols[2];
  DevCol* h_cols[2] = {nullptr, nullptr};
  size_t h_cols_cap[2] = {0, 0};
  // STR_IN lists per task (entries sorted by length, see TaskDesc)
  DevBuf<int32_t> d_list_i32;    // per task: start[kListLenSlots + 2], len[n], boff[n]
  DevBuf<uint64_t> d_list_pre;
  DevBuf<uint8_t> d_list_bytes;
  std::vector<int64_t> list_i32_base, list_pre_base, list_byte_base;
  ~dq_state() {
    for (int k = 0; k < 2; ++k) {
      if (h_tasks[k]) (void)hipHostFree(h_tasks[k]);
      if (h_cols[k]) (void)hipHostFree(h_cols[k]);
      if (h_order[k]) (void)hipHostFree(h_order[k]);
      if (ev[k]) (void)hipEventDestroy(ev[k]);
    }
    if (ev_xchg) (void)hipEventDestroy(ev_xchg);
  }
};

static void host_reset(dq_state* s) {
  const dq_plan* p = s->plan;
  s->acc.assign(p->tasks.size(), Acc{});
  for (size_t k = 0; k < p->tasks.size(); ++k) acc_init(p->tasks[k].kind, s->acc[k]);
  s->hll.assign((size_t)p->n_hll * kHllM, 0);
  s->rows = 0;
  s->host_dirty = true;
  s->synced = true;
}

// Pinned staging of at least `bytes` (the caller has set the device).
static dq_status pin_ensure(dq_state* s, size_t bytes) {
  if (s->h_pin_cap >= bytes) return DQ_OK;
  if (s->pin_pending) {
    HIP_TRY(host_wait(s->stream));
    s->pin_pending = false;
  }
  if (s->h_pin) (void)hipHostFree(s->h_pin);
  s->h_pin = nullptr;
  s->h_pin_cap = 0;
  HIP_TRY(hipHostMalloc(&s->h_pin, bytes, hipHostMallocDefault));
  s->h_pin_cap = bytes;
  return DQ_OK;
}

static dq_status upload_host(dq_state* s) {
  if (!s->host_dirty || s->device < 0) return DQ_OK;
  s->reset_pending = false;  // (the uploaded mirror is the device's base from here on)
  HIP_TRY(hipSetDevice(s->device));
  const size_t ab = s->acc.size() * sizeof(Acc), hb = s->hll.size();
  if (!s->stream_set) {  // no stream yet: blocking copies (the first scan may use any stream)
    if (ab) HIP_TRY(hipMemcpy(s->d_acc.p, s->acc.data(), ab, hipMemcpyHostToDevice));
    if (hb) HIP_TRY(hipMemcpy(s->d_hll.p, s->hll.data(), hb, hipMemcpyHostToDevice));
    HIP_TRY(hipMemsetAsync(s->d_queue.p, 0, kQueueWords * sizeof(uint32_t), nullptr));
    HIP_TRY(hipMemsetAsync(s->d_hll_stage.p, 0, s->d_hll_stage.n * sizeof(uint32_t), nullptr));
    HIP_TRY(host_wait(nullptr));  // the first scan may run on a non-blocking stream
    s->host_dirty = false;
    return DQ_OK;
  }
  // on the state's stream, ordered before the next scan: no host wait
  if (s->pin_pending) HIP_TRY(host_wait(s->stream));  // h_pin is about to be rewritten
  s->pin_pending = false;
  {
    const dq_status ps = pin_ensure(s, ab + hb);
    if (ps != DQ_OK) return ps;
  }
  uint8_t* pin = static_cast<uint8_t*>(s->h_pin);
  if (ab) {
    memcpy(pin, s->acc.data(), ab);
    HIP_TRY(hipMemcpyAsync(s->d_acc.p, pin, ab, hipMemcpyHostToDevice, s->stream));
  }
  if (hb) {
    memcpy(pin + ab, s->hll.data(), hb);
    HIP_TRY(hipMemcpyAsync(s->d_hll.p, pin + ab, hb, hipMemcpyHostToDevice, s->stream));
  }
  s->pin_pending = ab + hb > 0;
  HIP_TRY(hipMemsetAsync(s->d_queue.p, 0, kQueueWords * sizeof(uint32_t), s->stream));
  HIP_TRY(hipMemsetAsync(s->d_hll_stage.p, 0, s->d_hll_stage.n * sizeof(uint32_t), s->stream));
  s->host_dirty = false;
  return DQ_OK;
}

// The fused automaton of a regex blob (regex.py CompiledRegex.blob: int32 n_states, n_classes,
// start, 0; u8 class[256]; u8 status[n_states] padded to 4; u16 next[n_states * n_classes], the
// last class being end-of-text): u8 successor[state][byte] with the classes folded in and terminal
// states (status 1 sticky accept, 2 dead) made self-loops, then one flag byte per state -- bit 0:
// accepted once the end-of-text symbol is read from it, bit 1: terminal.  False when the automaton
// does not fit u8 states (the interpreter walks it instead).
static bool build_regex_table(const std::string& pool, int64_t at, std::vector<uint8_t>& tab,
                              int* ns_out, int* start_out) {
  if (at < 0 || (size_t)at + 16 + 256 > pool.size()) return false;
  const uint8_t* blob = reinterpret_cast<const uint8_t*>(pool.data()) + at;
  int32_t head[4];
  memcpy(head, blob, sizeof(head));
  const int ns = head[0], nc = head[1], start = head[2];
  if (ns < 1 || ns > kRegexMaxStates || nc < 2 || start < 0 || start >= ns) return false;
  const size_t nx_at = 16 + 256 + (size_t)((ns + 3) & ~3);
  if ((size_t)at + nx_at + (size_t)ns * nc * 2 > pool.size()) return false;
  const uint8_t* cls = blob + 16;
  const uint8_t* status = blob + 16 + 256;
  auto nx = [&](int q, int c) {
    uint16_t v;
    memcpy(&v, blob + nx_at + ((size_t)q * nc + c) * 2, 2);
    return (int)v;
  };
  tab.assign((size_t)ns * 257, 0);
  for (int q = 0; q < ns; ++q) {
    for (int b = 0; b < 256; ++b) {
      const int t = status[q] ? q : nx(q, cls[b]);
      if (t < 0 || t >= ns || cls[b] >= nc - 1) return false;
      tab[(size_t)q * 256 + b] = (uint8_t)t;
    }
    const int e = status[q] ? q : nx(q, nc - 1);
    if (e < 0 || e >= ns) return false;
    tab[(size_t)ns * 256 + q] = (uint8_t)((status[e] == 1 ? 1u : 0u) | (status[q] ? 2u : 0u));
  }
  *ns_out = ns;
  *start_out = start;
  return true;
}

extern "C" dq_status dq_state_create(const dq_plan* plan, int device, dq_state** out) {
  if (!plan || !out) return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  *out = nullptr;
  auto s = std::make_unique<dq_state>();
  s->plan = plan;
  s->device = device;
  host_reset(s.get());
  if (device < 0) {  // host-only state: deserialize / merge / get (rank-ordered merges)
    s->host_dirty = false;
    *out = s.release();
    return DQ_OK;
  }
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(DQ_ERR_DEVICE, "no HIP device %d", device);
  HIP_TRY(hipSetDevice(device));
  int cus = 0;
  HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
  for (int c = 0; c < kQueues; ++c) s->grid[c] = 0;
  for (const TaskPlan& t : plan->tasks) {
    const int c = body_class(plan, t);
    if (!s->grid[c]) s->grid[c] = std::max(1, cus * std::min(scan_max_blocks_per_cu(c, plan->n_hll), 8));
  }
  // the mixed launch also carries the HLL items when their LDS registers fit beside it
  s->mix_hll = plan->n_hll <= kMixedHllMax ? plan->n_hll : 0;
  s->grid[kBodyMixed] =
      std::max(1, cus * std::min(scan_max_blocks_per_cu(kBodyMixed, s->mix_hll), 8));
  const size_t nt = std::max<size_t>(1, plan->tasks.size());
  HIP_TRY(s->d_acc.ensure(nt));
  HIP_TRY(s->d_hll.ensure(std::max(1, plan->n_hll) * (size_t)kHllM));
  HIP_TRY(s->d_hll_stage.ensure(std::max(1, plan->n_hll) * (size_t)kHllM));
  HIP_TRY(s->d_queue.ensure(kQueueWords));
  HIP_TRY(s->d_partial.ensure(1024));
  HIP_TRY(s->d_partial2.ensure(nt * (size_t)kFinParts));
  HIP_TRY(s->d_fin_arrivals.ensure(nt));
  HIP_TRY(hipMemset(s->d_fin_arrivals.p, 0, nt * sizeof(uint32_t)));
  for (int k = 0; k < 2; ++k) HIP_TRY(hipEventCreateWithFlags(&s->ev[k], hipEventDisableTiming));
  HIP_TRY(hipEventCreateWithFlags(&s->ev_xchg, hipEventDisableTiming));
  // expression programs and string pools
  std::vector<XInstr> prog;
  std::string pool;
  for (const MatExpr& m : plan->mat) {
    s->prog_off.push_back((int)prog.size());
    prog.insert(prog.end(), m.prog.begin(), m.prog.end());
    while (pool.size() % 16) pool.push_back('\0');
    s->pool_off.push_back((int64_t)pool.size());
    pool += m.pool;
  }
  // PatternMatch over a utf8 column: its fused automaton table appended to the pool
  s->rx.assign(plan->mat.size(), dq_state::RegexRun{});
  for (size_t k = 0; k < plan->mat.size(); ++k) {
    std::vector<uint8_t> tab;
    int ns = 0, start = 0;
    const std::vector<XInstr>& pr = plan->mat[k].prog;
    if (pr.size() == 2 && pr[0].op == XI_COL && pr[1].op == XI_REGEX && pr[0].a >= 0 &&
        pr[0].a < (int)plan->types.size() && plan->types[pr[0].a] == DQ_UTF8 &&
        build_regex_table(plan->mat[k].pool, pr[1].imm, tab, &ns, &start)) {
      while (pool.size() % 16) pool.push_back('\0');
      s->rx[k] = dq_state::RegexRun{pr[0].a, pr[1].a, ns, start, (int64_t)pool.size()};
      pool.append(reinterpret_cast<const char*>(tab.data()), tab.size());
    }
  }
  // pool offsets in the programs are relative to each expression's own pool
  for (size_t k = 0; k < plan->mat.size(); ++k)
    for (size_t q = 0; q < plan->mat[k].prog.size(); ++q)
      if (prog[s->prog_off[k] + q].op == XI_STR || prog[s->prog_off[k] + q].op == XI_REGEX)
        prog[s->prog_off[k] + q].imm += s->pool_off[k];
  HIP_TRY(s->d_prog.ensure(std::max<size_t>(1, prog.size())));
  if (!prog.empty())
    HIP_TRY(hipMemcpy(s->d_prog.p, prog.data(), prog.size() * sizeof(XInstr), hipMemcpyHostToDevice));
  HIP_TRY(s->d_pool.ensure(std::max<size_t>(16, pool.size() + 16)));
  if (!pool.empty()) HIP_TRY(hipMemcpy(s->d_pool.p, pool.data(), pool.size(), hipMemcpyHostToDevice));
  // STR_IN lists: entries sorted by byte length and bucketed (TaskDesc::list_start)
  std::vector<int32_t> li32;
  std::vector<uint64_t> lpre;
  std::vector<uint8_t> lbytes;
  for (const TaskPlan& t : plan->tasks) {
    s->list_i32_base.push_back((int64_t)li32.size());
    s->list_pre_base.push_back((int64_t)lpre.size());
    s->list_byte_base.push_back((int64_t)lbytes.size());
    if (t.kind != TK_STR_IN) continue;
    std::vector<std::string> items = t.str.list;
    std::stable_sort(items.begin(), items.end(),
                     [](const std::string& a, const std::string& b) { return a.size() < b.size(); });
    // start[L] = number of entries whose bucket (length, or kListLenSlots when > 64) is < L, so
    // bucket L holds entries [start[L], start[L + 1])
    std::vector<int32_t> start(kListLenSlots + 2, 0);
    for (int L = 0; L < kListLenSlots + 2; ++L)
      for (const std::string& it : items)
        start[L] += ((it.size() <= 64 ? (int)it.size() : kListLenSlots) < L) ? 1 : 0;
    li32.insert(li32.end(), start.begin(), start.end());
    std::vector<int32_t> lens, boffs;
    for (const std::string& it : items) {
      lens.push_back((int32_t)it.size());
      boffs.push_back((int32_t)(lbytes.size() - s->list_byte_base.back()));
      uint64_t pre = 0;
      for (size_t b = 0; b < std::min<size_t>(8, it.size()); ++b)
        pre |= (uint64_t)(uint8_t)it[b] << (8 * b);
      lpre.push_back(pre);
      lbytes.insert(lbytes.end(), it.begin(), it.end());
    }
    li32.insert(li32.end(), lens.begin(), lens.end());
    li32.insert(li32.end(), boffs.begin(), boffs.end());
  }
  lbytes.resize(lbytes.size() + 16, 0);  // unaligned 8-byte reads past an entry's end stay inside
  HIP_TRY(s->d_list_i32.ensure(std::max<size_t>(1, li32.size())));
  HIP_TRY(s->d_list_pre.ensure(std::max<size_t>(1, lpre.size())));
  HIP_TRY(s->d_list_bytes.ensure(lbytes.size()));
  if (!li32.empty())
    HIP_TRY(hipMemcpy(s->d_list_i32.p, li32.data(), li32.size() * 4, hipMemcpyHostToDevice));
  if (!lpre.empty())
    HIP_TRY(hipMemcpy(s->d_list_pre.p, lpre.data(), lpre.size() * 8, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(s->d_list_bytes.p, lbytes.data(), lbytes.size(), hipMemcpyHostToDevice));
  dq_status st = upload_host(s.get());
  if (st != DQ_OK) return st;
  *out = s.release();
  return DQ_OK;
}

extern "C" void dq_state_destroy(dq_state* state) {
  if (!state) return;
  if (state->stream_set && state->device >= 0) (void)host_wait(state->stream);
  if (state->h_pin) (void)hipHostFree(state->h_pin);
  delete state;
}

extern "C" dq_status dq_state_reset(dq_state* state) {
  if (!state) return fail(DQ_ERR_INVALID_ARGUMENT, "null state");
  if (state->stream_set && state->device >= 0) HIP_TRY(host_wait(state->stream));
  host_reset(state);
  static const bool eager = getenv("DQ_EAGER_RESET") != nullptr;  // A/B hook
  if (state->stream_set && state->device >= 0 && !eager) {
    state->host_dirty = false;  // (the device words are ignored until the next scan rewrites them)
    state->reset_pending = true;
    state->rows_on_device = false;
    return DQ_OK;
  }
  return upload_host(state);
}

static int64_t pow2_at_least(int64_t v) {
  int64_t p = 1;
  while (p < v) p <<= 1;
  return p;
}

static bool aligned(const void* p, uintptr_t a) { return (reinterpret_cast<uintptr_t>(p) & (a - 1)) == 0; }



namespace dq {
// What a plan reads of each column: 0 nothing, 1 the validity bitmap only (Completeness: a
// TK_VALIDITY task), 2 every buffer.  The columnar loader stages only that (loader.cpp).
void plan_column_needs(const dq_plan* plan, std::vector<int>& need) {
  need.assign(plan->types.size(), 0);
  for (const TaskPlan& t : plan->tasks) {
    const int v = t.kind == TK_VALIDITY ? 1 : 2;
    if (t.col >= 0) need[t.col] = std::max(need[t.col], v);
    if (t.col2 >= 0) need[t.col2] = std::max(need[t.col2], v);
  }
  for (const MatExpr& m : plan->mat)
    for (const XInstr& ins : m.prog)
      if (ins.op == XI_COL) need[ins.a] = 2;
}
}  // namespace dq

// Validates one batch against the plan and returns its row count (-1 on error).
static int64_t batch_rows(const dq_plan* plan, const dq_column* cols, const std::vector<int>& ref,
                          dq_status& st) {
  st = DQ_OK;
  int64_t rows = -1;
  for (size_t c = 0; c < plan->types.size(); ++c) {
    if (cols[c].type != plan->types[c]) {
      st = fail(DQ_ERR_WRONG_TYPE, "column %zu has type %d, plan expects %d", c, cols[c].type,
                plan->types[c]);
      return -1;
    }
    if (!ref[c]) continue;
    if (cols[c].length < 0) {
      st = fail(DQ_ERR_INVALID_ARGUMENT, "negative column length");
      return -1;
    }
    if (rows < 0) rows = cols[c].length;
    else if (rows != cols[c].length) {
      st = fail(DQ_ERR_INVALID_ARGUMENT, "columns of one batch differ in length");
      return -1;
    }
    if (cols[c].length > 0 && !cols[c].values) {
      st = fail(DQ_ERR_INVALID_ARGUMENT, "column %zu has no values buffer", c);
      return -1;
    }
    if (cols[c].type == DQ_UTF8 && cols[c].length > 0 && !cols[c].data) {
      st = fail(DQ_ERR_INVALID_ARGUMENT, "utf8 column %zu has no data buffer", c);
      return -1;
    }
  }
  if (rows < 0) rows = plan->types.empty() ? 0 : cols[0].length;  // e.g. only Size()
  if (rows > ((int64_t)1 << 40)) {
    st = fail(DQ_ERR_UNSUPPORTED, "batch too large");
    return -1;
  }
  return rows;
}

extern "C" dq_status dq_scan_device(const dq_plan* plan, const dq_column* cols, int n_cols,
                                    dq_state* s, void* hip_stream) {
  return dq_scan_device_batches(plan, cols, n_cols, 1, s, hip_stream);
}

// ---- guided tail of the scan queue ----------------------------------------------------------
constexpr int64_t kTailDiv = 32;      // the last 1/32 of a descriptor's items ...
constexpr int64_t kTailCut = 8;       // ... are cut 8 ways
constexpr int64_t kTailMinItems = 16;
static bool tail_split() {  // DQ_TAIL_SPLIT=0: A/B hook, uniform items
  static const bool on = [] {
    const char* e = getenv("DQ_TAIL_SPLIT");
    return !e || atoi(e) != 0;
  }();
  return on;
}

// Does launch L (one class, items [item_lo, item_hi)) have small tail items?
static bool scan_has_tail(const TaskDesc* td, size_t n_desc, const ScanLaunch& L) {
  for (size_t q = 0; q < n_desc; ++q)
    if (td[q].n_items > td[q].n_big && (uint32_t)td[q].item_begin >= L.item_lo &&
        (uint32_t)td[q].item_begin < L.item_hi)
      return true;
  return false;
}

// The queue order of the launches of one queue (one class, or the classes of a mixed launch),
// appended to `out`: within the big items and within the small ones, the classes interleaved in
// proportion to their counts; then each of the kernel's kQueueHeads slices (queue_next: entries
// [n x / H, n (x + 1) / H)) is filled with its share of the big items followed by its share of
// the small ones, so every slice ends on small items.
static void scan_order(const TaskDesc* td, size_t n_desc, const std::vector<ScanLaunch>& G,
                       std::vector<uint32_t>& out) {
  std::vector<std::vector<uint32_t>> big(G.size()), small(G.size());
  for (size_t c = 0; c < G.size(); ++c)
    for (size_t q = 0; q < n_desc; ++q) {
      const TaskDesc& t = td[q];
      if (t.n_items == 0 || (uint32_t)t.item_begin < G[c].item_lo || (uint32_t)t.item_begin >= G[c].item_hi)
        continue;
      for (int64_t i = 0; i < t.n_items; ++i)
        (i < t.n_big ? big[c] : small[c]).push_back((uint32_t)(t.item_begin + i));
    }
  auto interleave = [](std::vector<std::vector<uint32_t>>& lists) {
    std::vector<uint32_t> r;
    std::vector<size_t> next(lists.size(), 0);
    size_t total = 0;
    for (auto& l : lists) total += l.size();
    r.reserve(total);
    for (size_t k = 0; k < total; ++k) {
      int best = -1;
      double best_key = 0.0;
      for (size_t c = 0; c < lists.size(); ++c) {
        if (next[c] >= lists[c].size()) continue;
        const double key = (next[c] + 0.5) / (double)lists[c].size();
        if (best < 0 || key < best_key) {
          best = (int)c;
          best_key = key;
        }
      }
      r.push_back(lists[best][next[best]++]);
    }
    return r;
  };
  const std::vector<uint32_t> B = interleave(big), S = interleave(small);
  const uint64_t n = B.size() + S.size();
  size_t bi = 0, si = 0;
  for (int x = 0; x < kQueueHeads; ++x) {
    const uint64_t len = n * (x + 1) / kQueueHeads - n * x / kQueueHeads;
    const uint64_t want_s = (uint64_t)S.size() * (x + 1) / kQueueHeads - (uint64_t)si;
    uint64_t ns = std::min<uint64_t>(want_s, len), nb = len - ns;
    if (nb > B.size() - bi) {  // (rounding: not enough big items left, take small ones)
      nb = B.size() - bi;
      ns = len - nb;
    }
    for (uint64_t k = 0; k < nb; ++k) out.push_back(B[bi++]);
    for (uint64_t k = 0; k < ns; ++k) out.push_back(S[si++]);
  }
}

extern "C" dq_status dq_scan_device_batches(const dq_plan* plan, const dq_column* cols, int n_cols,
                                            int n_batches, dq_state* s, void* hip_stream) {
  if (!plan || !s || (n_cols > 0 && n_batches > 0 && !cols))
    return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  if (n_batches < 0) return fail(DQ_ERR_INVALID_ARGUMENT, "negative batch count");
  if (s->plan != plan) return fail(DQ_ERR_STATE, "state was created for another plan");
  if (n_cols < (int)plan->types.size())
    return fail(DQ_ERR_NO_SUCH_COLUMN, "plan needs %zu columns, got %d", plan->types.size(), n_cols);
  if (n_batches == 0) return DQ_OK;
  if (s->device < 0) return fail(DQ_ERR_STATE, "host-only state (device -1) cannot scan");
  hipStream_t stream = reinterpret_cast<hipStream_t>(hip_stream);
  HIP_TRY(hipSetDevice(s->device));
  if (s->rows_on_device) {  // an exchange's merged rows: read back before adding to them
    const dq_status rs = dq_state_sync(s);
    if (rs != DQ_OK) return rs;
  }
  if (s->stream_set && s->stream != stream) HIP_TRY(host_wait(s->stream));
  s->stream = stream;
  s->stream_set = true;
  dq_status st = upload_host(s);
  if (st != DQ_OK) return st;

  // referenced columns decide each batch's length
  std::vector<int> ref(plan->types.size(), 0);
  for (const TaskPlan& t : plan->tasks) {
    if (t.col >= 0) ref[t.col] = 1;
    if (t.col2 >= 0) ref[t.col2] = 1;
  }
  for (const MatExpr& m : plan->mat)
    for (const XInstr& ins : m.prog)
      if (ins.op == XI_COL) ref[ins.a] = 1;
  std::vector<int64_t> rows(n_batches);
  int64_t total_rows = 0;
  for (int b = 0; b < n_batches; ++b) {
    rows[b] = batch_rows(plan, cols + (size_t)b * n_cols, ref, st);
    if (rows[b] < 0) return st;
    total_rows += rows[b];
  }

  const int slot = s->flip;
  s->flip ^= 1;
  if (s->ev_used[slot]) HIP_TRY(host_wait_event(s->ev[slot]));

  // materialised expressions -> bitmaps, per batch at a 16-byte aligned word offset
  std::vector<size_t> bm_off(n_batches);
  size_t words = 0;
  for (int b = 0; b < n_batches; ++b) {
    bm_off[b] = words;
    words += (size_t)((rows[b] + 63) / 64 + 2) & ~(size_t)1;
  }
  words += 2;
  const size_t n_mat = plan->mat.size();
  if (n_mat) {
    if (words > s->bitmap_words || !s->d_bitmaps.p) {
      HIP_TRY(host_wait(stream));
      HIP_TRY(s->d_bitmaps.ensure(words * 2 * n_mat));
      s->bitmap_words = words;
    }
    const size_t ncol = plan->types.size();
    HIP_TRY(s->d_cols[slot].ensure(std::max<size_t>(1, ncol * n_batches)));
    if (s->h_cols_cap[slot] < ncol * n_batches) {
      if (s->h_cols[slot]) HIP_TRY(hipHostFree(s->h_cols[slot]));
      HIP_TRY(hipHostMalloc((void**)&s->h_cols[slot], ncol * n_batches * sizeof(DevCol),
                            hipHostMallocDefault));
      s->h_cols_cap[slot] = ncol * n_batches;
    }
    DevCol* hc = s->h_cols[slot];
    for (int b = 0; b < n_batches; ++b)
      for (size_t c = 0; c < ncol; ++c) {
        const dq_column& col = cols[(size_t)b * n_cols + c];
        hc[b * ncol + c] = DevCol{col.type, 0, col.validity, col.values, col.data};
      }
    HIP_TRY(hipMemcpyAsync(s->d_cols[slot].p, hc, ncol * n_batches * sizeof(DevCol),
                           hipMemcpyHostToDevice, stream));
    for (size_t k = 0; k < n_mat; ++k) {
      for (int b = 0; b < n_batches; ++b) {
        uint64_t* val = s->d_bitmaps.p + (2 * k) * s->bitmap_words + bm_off[b];
        uint64_t* vld = s->d_bitmaps.p + (2 * k + 1) * s->bitmap_words + bm_off[b];
        const dq_state::RegexRun& rx = s->rx[k];
        if (rx.col >= 0) {
          const dq_column& col = cols[(size_t)b * n_cols + rx.col];
          HIP_TRY(launch_regex(col.validity, reinterpret_cast<const int32_t*>(col.values), col.data,
                               rows[b], s->d_pool.p + rx.table_off, rx.ns, rx.start, rx.null_mode,
                               val, vld, stream));
        } else {
          HIP_TRY(launch_expr(s->d_prog.p + s->prog_off[k], (int)plan->mat[k].prog.size(),
                              s->d_cols[slot].p + (size_t)b * ncol, s->d_pool.p, rows[b], val, vld,
                              stream));
        }
      }
    }
  }
  auto mat_val = [&](int m, int b) -> const uint8_t* {
    if (m < 0) return nullptr;
    return reinterpret_cast<const uint8_t*>(s->d_bitmaps.p + (2 * m) * s->bitmap_words + bm_off[b]);
  };
  auto mat_vld = [&](int m, int b) -> const uint8_t* {
    if (m < 0) return nullptr;
    return reinterpret_cast<const uint8_t*>(s->d_bitmaps.p + (2 * m + 1) * s->bitmap_words + bm_off[b]);
  };

  // descriptor table: one descriptor per (batch, task)
  const size_t n_desc = plan->tasks.size() * (size_t)n_batches;
  if (s->h_tasks_cap[slot] < n_desc) {
    if (s->h_tasks[slot]) HIP_TRY(hipHostFree(s->h_tasks[slot]));
    HIP_TRY(hipHostMalloc((void**)&s->h_tasks[slot], std::max<size_t>(1, n_desc) * sizeof(TaskDesc),
                          hipHostMallocDefault));
    s->h_tasks_cap[slot] = n_desc;
  }
  HIP_TRY(s->d_tasks[slot].ensure(std::max<size_t>(1, n_desc)));
  TaskDesc* td = s->h_tasks[slot];
  int64_t total_items = 0;
  size_t d = 0;
  // class-major, then task-major: the items of one body class form one launch, and the items of
  // one logical task one contiguous range (finalize relies on it)
  std::vector<ScanLaunch> launches;
  std::vector<size_t> order;
  for (int c = 0; c < kBodyClasses; ++c)
    for (size_t k = 0; k < plan->tasks.size(); ++k)
      if (body_class(plan, plan->tasks[k]) == c) order.push_back(k);
  for (size_t k : order) {
    const TaskPlan& tp = plan->tasks[k];
    for (int b = 0; b < n_batches; ++b, ++d) {
      const dq_column* bc = cols + (size_t)b * n_cols;
      TaskDesc t;
      memset(&t, 0, sizeof(t));
      t.kind = tp.kind;
      t.body = body_class(plan, tp);
      t.out = tp.out;
      t.hll_out = tp.kind == TK_COMOMENTS ? tp.fused_hll : tp.hll_out;
      t.hll_side = tp.hll_side;
      t.batch = b;
      t.rows = rows[b];
      t.w_val = mat_val(tp.where, b);
      t.w_vld = mat_vld(tp.where, b);
      // item sizing: ~128 KiB of the task's buffers per item (a few bodies weighted by work)
      double bpr = 0.0;
      bool vec = aligned(t.w_val, 16) && aligned(t.w_vld, 16);
      if (tp.col >= 0) {
        const dq_column& c = bc[tp.col];
        // an HLL task hashes a date as its int32 and a timestamp as its int64 (the bodies' fast
        // paths); every other body reads the column as its own type
        t.type = tp.kind == TK_HLL ? phys_type(c.type) : c.type;
        t.valid = c.validity;
        t.values = c.values;
        t.data = c.data;
        vec = vec && aligned(c.validity, 16) && aligned(c.values, 16);
        bpr += type_size(c.type) + 0.125;
        if (c.type == DQ_UTF8) bpr += 8.0;
      }
      if (tp.col2 >= 0) {
        const dq_column& c = bc[tp.col2];
        t.type2 = c.type;
        t.valid2 = c.validity;
        t.values2 = c.values;
        vec = vec && aligned(c.validity, 16) && aligned(c.values, 16);
        bpr += type_size(c.type) + 0.125;
      }
      switch (tp.kind) {
        case TK_NUMERIC:
          t.n_preds = tp.n_preds;
          for (int q = 0; q < tp.n_preds; ++q) t.preds[q] = tp.preds[q];
          break;
        case TK_BOOLMAP:
          t.b_val = mat_val(tp.bool_expr, b);
          t.b_vld = mat_vld(tp.bool_expr, b);
          vec = vec && aligned(t.b_val, 16) && aligned(t.b_vld, 16);
          bpr = 0.25;
          break;
        case TK_VALIDITY: bpr = 0.125; break;
        case TK_STR_IN: {
          t.negate = tp.str.negate ? 1 : 0;
          t.null_is_true = tp.str.null_is_true ? 1 : 0;
          t.n_list = (int32_t)tp.str.list.size();
          const int32_t* base = s->d_list_i32.p + s->list_i32_base[k];
          t.list_start = base;
          t.list_len = base + kListLenSlots + 2;
          t.list_boff = base + kListLenSlots + 2 + t.n_list;
          t.list_pre = s->d_list_pre.p + s->list_pre_base[k];
          t.list_bytes = s->d_list_bytes.p + s->list_byte_base[k];
          t.list_small = t.n_list <= 8 ? 1 : 0;
          t.list_lenmask = 0;
          for (int e = 0; e < 8; ++e) t.list_key[e] = 0xFEULL << 56;  // no row key has top byte 0xFE
          for (size_t e = 0; e < tp.str.list.size(); ++e) {
            const std::string& it = tp.str.list[e];
            if (it.size() > 7) {
              t.list_small = 0;
              continue;
            }
            t.list_lenmask |= 1ULL << it.size();
            if (e < 8) {
              uint64_t key = (uint64_t)it.size() << 56;
              for (size_t q = 0; q < it.size(); ++q) key |= (uint64_t)(uint8_t)it[q] << (8 * q);
              t.list_key[e] = key;
            }
          }
          break;
        }
        // (items of HLL / co-moment tasks were once sized by work -- 4x / 2x the bytes -- but
        // then the single dequeue word, ~88 dequeues/us, became the bound: items are sized by
        // bytes only)
        default: break;
      }
      if (tp.where >= 0) bpr += 0.25;
      t.vec_ok = vec ? 1 : 0;
      int64_t item_rows = pow2_at_least((int64_t)(kItemBytes / std::max(bpr, 1e-3)));
      item_rows = std::max<int64_t>(kItemAlign, std::min<int64_t>(item_rows, (int64_t)1 << 22));
      t.item_rows = item_rows;
      // a carried HLL task keeps its (empty) descriptors: finalize finds the task through them
      t.n_items = rows[b] > 0 && !tp.carried ? (rows[b] + item_rows - 1) / item_rows : 0;
      t.n_big = t.n_items;
      t.small_rows = item_rows;
      // guided tail: the last 1/kTailDiv of a descriptor's items are cut kTailCut ways; the queue
      // order hands these out last in every slice (scan_orders), so the waves of a launch finish
      // within a small item of each other instead of a ~130 us big item (S10: ~3000 waves)
      if (tail_split() && t.n_items >= kTailMinItems && item_rows >= kTailCut * kItemAlign) {
        const int64_t k = (t.n_items + kTailDiv - 1) / kTailDiv;
        t.n_big = t.n_items - k;
        t.small_rows = item_rows / kTailCut;
        t.n_items = t.n_big + (rows[b] - t.n_big * item_rows + t.small_rows - 1) / t.small_rows;
      }
      t.item_begin = total_items;
      total_items += t.n_items;
      td[d] = t;
    }
    const int c = body_class(plan, tp);
    if (launches.empty() || launches.back().body != c)
      launches.push_back(ScanLaunch{c, s->grid[c], (uint32_t)td[d - n_batches].item_begin, 0, nullptr});
    launches.back().item_hi = (uint32_t)total_items;
  }
  if (total_items >= ((int64_t)1 << 31))
    return fail(DQ_ERR_UNSUPPORTED, "scan of %lld work items exceeds one launch",
                (long long)total_items);
  // Queue orders.  Two or more body classes: one mixed launch over their items, interleaved in
  // proportion to each class's item count (item j of a class with n items sorts at (j + 1/2) / n),
  // so string gathers, XXH64 hashing and streaming bodies run side by side.  HLL joins the mixed
  // launch when its LDS registers fit (s->mix_hll), else it keeps its own launch.  A launch whose
  // descriptors have small tail items gets an order list too (scan_orders: big items, then the
  // small ones at the end of every queue slice).
  {
    std::vector<ScanLaunch> plain, hll;
    for (const ScanLaunch& L : launches)
      // the fused body keeps HLL registers in LDS too, and the mixed kernel has no such body
      ((L.body == BC_HLL && !s->mix_hll) || L.body == BC_CORR_HLL || L.body == BC_DECIMAL ? hll : plain)
          .push_back(L);
    const bool mixed = plain.size() >= 2 && !getenv("DQ_NO_MIXED");
    if (mixed && plain.front().item_lo != 0) return fail(DQ_ERR_STATE, "unexpected item layout");
    std::vector<std::vector<ScanLaunch>> groups;  // the launches that share one queue
    if (mixed) groups.push_back(plain);
    else
      for (const ScanLaunch& L : plain) groups.push_back({L});
    for (const ScanLaunch& L : hll) groups.push_back({L});
    std::vector<uint32_t> sig;
    for (size_t q = 0; q < n_desc; ++q) {
      sig.push_back((uint32_t)td[q].item_begin);
      sig.push_back((uint32_t)td[q].n_big);
      sig.push_back((uint32_t)td[q].n_items);
    }
    for (const auto& G : groups) {
      sig.push_back(0xffffffffu);
      for (const ScanLaunch& L : G) {
        sig.push_back(L.item_lo);
        sig.push_back(L.item_hi);
      }
    }
    // (built only when the descriptors change: ~1e5 items per S10 step, cached per slot)
    std::vector<size_t>& off = s->order_off[slot];
    std::vector<size_t>& len = s->order_len[slot];
    if (s->order_sig[slot] != sig) {
      off.assign(groups.size(), 0);
      len.assign(groups.size(), 0);
      std::vector<uint32_t> all;
      for (size_t g = 0; g < groups.size(); ++g) {
        off[g] = all.size();
        if (groups[g].size() >= 2 || scan_has_tail(td, n_desc, groups[g][0])) {
          scan_order(td, n_desc, groups[g], all);
          len[g] = all.size() - off[g];
        }
      }
      HIP_TRY(s->d_order[slot].ensure(std::max<size_t>(1, all.size())));
      if (!all.empty()) {
        // staged in the slot's pinned buffer and queued on `stream`: the slot's event was waited
        // above, so neither buffer is still read, and the other slot's work is not waited for
        if (s->h_order_cap[slot] < all.size()) {
          if (s->h_order[slot]) HIP_TRY(hipHostFree(s->h_order[slot]));
          s->h_order[slot] = nullptr;
          s->h_order_cap[slot] = 0;
          HIP_TRY(hipHostMalloc((void**)&s->h_order[slot], all.size() * sizeof(uint32_t),
                                hipHostMallocDefault));
          s->h_order_cap[slot] = all.size();
        }
        memcpy(s->h_order[slot], all.data(), all.size() * sizeof(uint32_t));
        HIP_TRY(hipMemcpyAsync(s->d_order[slot].p, s->h_order[slot], all.size() * sizeof(uint32_t),
                               hipMemcpyHostToDevice, stream));
      }
      s->order_sig[slot] = sig;
    }
    launches.clear();
    for (size_t g = 0; g < groups.size(); ++g) {
      const uint32_t* ord = len[g] ? s->d_order[slot].p + off[g] : nullptr;
      if (groups[g].size() >= 2) {
        bool has_hll = false;
        uint32_t classes = 0;
        for (const ScanLaunch& L : groups[g]) {
          has_hll = has_hll || L.body == BC_HLL;
          classes |= 1u << L.body;
        }
        launches.push_back(ScanLaunch{kBodyMixed, s->grid[kBodyMixed], 0, (uint32_t)len[g], ord,
                                      has_hll ? s->mix_hll : 0, classes});
      } else {
        ScanLaunch L = groups[g][0];
        if (ord) {
          L.item_lo = 0;
          L.item_hi = (uint32_t)len[g];
          L.order = ord;
        }
        launches.push_back(L);
      }
    }
  }
  if (getenv("DQ_DEBUG")) {
    for (const ScanLaunch& L : launches)
      fprintf(stderr, "[dq] launch body=%d grid=%d items=[%u,%u)\n", L.body, L.grid, L.item_lo,
              L.item_hi);
    for (size_t q = 0; q < n_desc; ++q)
      fprintf(stderr, "[dq] desc %zu kind=%d out=%d rows=%lld item_rows=%lld items=[%lld,+%lld) vec=%d\n",
              q, td[q].kind, td[q].out, (long long)td[q].rows, (long long)td[q].item_rows,
              (long long)td[q].item_begin, (long long)td[q].n_items, td[q].vec_ok);
  }
  if (n_desc > 0 && total_items > 0) {
    HIP_TRY(s->d_partial.ensure((size_t)total_items));
    HIP_TRY(hipMemcpyAsync(s->d_tasks[slot].p, td, n_desc * sizeof(TaskDesc), hipMemcpyHostToDevice,
                           stream));
    HIP_TRY(launch_scan(s->d_tasks[slot].p, (int)n_desc, (int)plan->tasks.size(), launches.data(),
                        (int)launches.size(), plan->n_hll, s->d_queue.p, s->d_partial.p,
                        s->d_partial2.p, s->d_hll_stage.p, s->d_acc.p, s->d_hll.p,
                        s->d_fin_arrivals.p, stream, s->reset_pending ? 1 : 0));
    s->reset_pending = false;
    s->synced = false;
  }
  HIP_TRY(hipEventRecord(s->ev[slot], stream));
  s->ev_used[slot] = true;
  s->rows += total_rows;
  return DQ_OK;
}

extern "C" dq_status dq_state_sync(dq_state* s) {
  if (!s) return fail(DQ_ERR_INVALID_ARGUMENT, "null state");
  if (s->synced || s->device < 0) return DQ_OK;
  HIP_TRY(hipSetDevice(s->device));
  // both read-backs queued behind the scan on its stream, one host wait
  const size_t ab = s->acc.size() * sizeof(Acc), hb = s->hll.size();
  const size_t rb = s->rows_on_device ? 8 : 0;
  {
    const dq_status ps = pin_ensure(s, ab + hb + 8);
    if (ps != DQ_OK) return ps;
  }
  uint8_t* pin = static_cast<uint8_t*>(s->h_pin);
  if (ab) HIP_TRY(hipMemcpyAsync(pin, s->d_acc.p, ab, hipMemcpyDeviceToHost, s->stream));
  if (hb) HIP_TRY(hipMemcpyAsync(pin + ab, s->d_hll.p, hb, hipMemcpyDeviceToHost, s->stream));
  if (rb) HIP_TRY(hipMemcpyAsync(pin + ab + hb, s->d_rows.p, rb, hipMemcpyDeviceToHost, s->stream));
  HIP_TRY(host_wait(s->stream));
  s->pin_pending = false;
  if (ab) memcpy(s->acc.data(), pin, ab);
  if (hb) memcpy(s->hll.data(), pin + ab, hb);
  if (rb) memcpy(&s->rows, pin + ab + hb, 8);
  s->rows_on_device = false;
  s->synced = true;
  return DQ_OK;
}

static void pack_hll(const uint8_t* regs, uint64_t* words) {
  for (int w = 0; w < kHllWords; ++w) {
    uint64_t v = 0;
    for (int i = 0; i < kHllRegsPerWord; ++i) {
      int idx = w * kHllRegsPerWord + i;
      if (idx >= kHllM) break;
      v |= (uint64_t)(regs[idx] & 0x3f) << (kHllRegBits * i);
    }
    words[w] = v;
  }
}

extern "C" dq_status dq_state_get(const dq_state* s, int agg_index, dq_value* out) {
  if (!s || !out) return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  const dq_plan* p = s->plan;
  if (agg_index < 0 || agg_index >= (int)p->slots.size())
    return fail(DQ_ERR_INVALID_ARGUMENT, "aggregation index %d out of range", agg_index);
  if (!s->synced) return fail(DQ_ERR_STATE, "state not synced (call dq_state_sync)");
  memset(out, 0, sizeof(*out));
  const Slot& sl = p->slots[agg_index];
  out->kind = sl.kind;
  if (sl.src == SRC_ROWS) {
    out->i64 = s->rows;
    out->f64[0] = (double)s->rows;
    return DQ_OK;
  }
  const TaskPlan& tp = p->tasks[sl.task];
  const Acc& a = s->acc[sl.task];
  switch (sl.kind) {
    case DQ_AGG_COUNT_NOTNULL:
      out->i64 = tp.kind == TK_NUMERIC ? a.i[0] : a.i[0];
      out->is_null = s->rows == 0;
      break;
    case DQ_AGG_COUNT_TRUE:
      if (sl.fused_pred) {
        out->i64 = a.i[4 + sl.field];
        out->is_null = a.i[7 + sl.field] == 0;
      } else {
        out->i64 = a.i[0];
        out->is_null = a.i[1] == 0;
      }
      break;
    case DQ_AGG_SUM:
      out->is_null = a.i[0] == 0;
      if (is_decimal(sl.col_type)) {  // exact sum; NULL when it overflows the result type
        for (int q = 0; q < 3; ++q) out->words[q] = (uint64_t)a.i[1 + q];
        out->words[3] = a.i[3] < 0 ? ~0ULL : 0ULL;
        if (!out->is_null && !dec_sum_fits((uint64_t)a.i[1], (uint64_t)a.i[2], (uint64_t)a.i[3],
                                           DQ_DECIMAL_PRECISION(sl.col_type)))
          out->is_null = 1;
        out->f64[0] = out->is_null ? 0.0
                                   : dec192_to_double((uint64_t)a.i[1], (uint64_t)a.i[2],
                                                      (uint64_t)a.i[3], DQ_DECIMAL_SCALE(sl.col_type));
      } else if (is_integral(sl.col_type)) {
        out->i64 = a.i[1];
        out->f64[0] = (double)a.i[1];
      } else {
        out->f64[0] = a.d[0];
      }
      break;
    case DQ_AGG_MIN:
    case DQ_AGG_MAX: {
      out->is_null = a.i[0] == 0;
      if (is_decimal(sl.col_type)) {
        const int at = sl.kind == DQ_AGG_MIN ? 4 : 6;
        out->words[0] = (uint64_t)a.i[at];
        out->words[1] = (uint64_t)a.i[at + 1];
        out->f64[0] = out->is_null ? 0.0
                                   : dec_to_double((uint64_t)a.i[at], a.i[at + 1],
                                                   DQ_DECIMAL_SCALE(sl.col_type));
        break;
      }
      int64_t k = sl.kind == DQ_AGG_MIN ? a.i[2] : a.i[3];
      if (is_integral(sl.col_type)) {
        out->i64 = k;
        out->f64[0] = (double)k;
      } else {
        out->f64[0] = f64_from_key(k);
      }
      break;
    }
    case DQ_AGG_STDDEV_POP:
      out->f64[0] = (double)a.i[0];
      out->f64[1] = a.i[0] ? a.d[1] : 0.0;
      out->f64[2] = a.i[0] ? a.d[2] : 0.0;
      break;
    case DQ_AGG_CORR:
      out->f64[0] = (double)a.i[0];
      for (int f = 0; f < 5; ++f) out->f64[1 + f] = a.i[0] ? a.d[f] : 0.0;
      break;
    case DQ_AGG_HLL:
      pack_hll(&s->hll[(size_t)tp.hll_out * kHllM], out->words);
      break;
    case DQ_AGG_DTYPE:  // the UDAF's buffer is never NULL (StatefulDataType.initialize)
      for (int q = 0; q < 5; ++q) out->words[q] = (uint64_t)a.i[q];
      break;
    default: break;
  }
  return DQ_OK;
}

extern "C" dq_status dq_state_get_all(const dq_state* s, int n, dq_value* out) {
  if (!s || (!out && n > 0)) return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  for (int k = 0; k < n; ++k) {
    const dq_status st = dq_state_get(s, k, out + k);
    if (st != DQ_OK) return st;
  }
  return DQ_OK;
}

// ------------------------------------------------------------------------------------------------
// State exchange across ranks (distributed.py exchange_states): the counters and
// wrapping Long sums meet in ONE SUM all-reduce, the extremes in ONE MAX all-reduce, the HLL
// registers (u8) in ONE MAX all-reduce, and the fp64 moments in ONE all-gather that a kernel merges
// in rank order with acc_merge's rules (StandardDeviation.scala:37-44, Correlation.scala:37-52).
// The result equals dq_state_merge over the ranks' states in rank order, bit for bit: integer adds
// wrap and are associative, max / min are exact, and the fp64 merges run in the same order from
// the same inputs.
//   isum[10 T + 1]   every task's Acc.i (TK_NUMERIC's min / max keys and TK_DECIMAL's 128-bit
//                    words as 0), then the rows
//   imax[2 T]        TK_NUMERIC max keys, then ~min keys (bitwise NOT reverses the signed order:
//                    MAX of ~min = ~MIN)
//   hll[512 n_hll]   the HLL registers (StatefulHyperloglogPlus.scala:119-137 merges by max)
//   mom[16 T]        per task: n, 1 when acc_merge would not skip the buffer, d0..d5, then (TK_DECIMAL)
//                    its i1..i7 as raw bits -- the 192-bit sum and 128-bit extremes, whose carries
//                    and lexicographic order no word-wise collective keeps -- merged in rank order
//                    by acc_merge; gathered rank-major as [world][16 T]
// The task kinds live on the device from the state's first exchange (plans are immutable): no
// upload and no host wait per call.
// ------------------------------------------------------------------------------------------------
namespace {
constexpr int kMomW = 16;

DQ_HD void xchg_pack_task(int kind, const Acc& a, int k, int T, int64_t* isum, int64_t* imax,
                          double* mom) {
  for (int q = 0; q < 10; ++q) isum[10 * k + q] = a.i[q];
  if (kind == TK_NUMERIC) {
    isum[10 * k + 2] = isum[10 * k + 3] = 0;
    imax[k] = a.i[3];
    imax[T + k] = ~a.i[2];
  } else {
    imax[k] = imax[T + k] = INT64_MIN;
  }
  double* m = mom + (size_t)kMomW * k;
  const bool live = kind == TK_NUMERIC ? (a.i[0] || a.i[7] || a.i[8] || a.i[9]) : a.i[0] != 0;
  m[0] = (double)a.i[0];
  m[1] = live ? 1.0 : 0.0;
  for (int q = 0; q < 6; ++q) m[2 + q] = a.d[q];
  for (int q = 8; q < kMomW; ++q) m[q] = 0.0;
  if (kind == TK_DECIMAL) {
    for (int q = 1; q < 8; ++q) {
      isum[10 * k + q] = 0;
      m[7 + q] = __builtin_bit_cast(double, a.i[q]);
    }
  }
}

// The merged Acc of task k: acc_merge(init, rank 0, rank 1, ...) restated over the exchange
DQ_HD void xchg_merge_task(int kind, int k, int T, int world, const int64_t* isum,
                           const int64_t* imax, const double* momg, Acc& out) {
  if (kind == TK_DECIMAL) {  // every field from the gathered words, in rank order
    acc_init(kind, out);
    for (int r = 0; r < world; ++r) {
      const double* b = momg + ((size_t)r * T + k) * kMomW;
      Acc a;
      acc_init(kind, a);
      a.i[0] = (int64_t)b[0];
      for (int q = 1; q < 8; ++q) a.i[q] = __builtin_bit_cast(int64_t, b[7 + q]);
      for (int q = 0; q < 6; ++q) a.d[q] = b[2 + q];
      acc_merge(kind, out, a);
    }
    return;
  }
  for (int q = 0; q < 10; ++q) out.i[q] = isum[10 * k + q];
  for (int q = 0; q < 6; ++q) out.d[q] = 0.0;
  if (kind == TK_NUMERIC) {
    out.i[2] = ~imax[T + k];
    out.i[3] = imax[k];
  }
  double na = 0.0;
  for (int r = 0; r < world; ++r) {
    const double* b = momg + ((size_t)r * T + k) * kMomW;
    if (kind == TK_NUMERIC) {
      if (b[1] == 0.0) continue;
      if (b[0] > 0.0) {
        if (na == 0.0) {
          out.d[1] = b[3];
          out.d[2] = b[4];
        } else {
          moments_merge(na, out.d[1], out.d[2], b[0], b[3], b[4]);
        }
      }
      na += b[0];
      out.d[0] += b[2];
    } else if (kind == TK_COMOMENTS) {
      if (b[0] == 0.0) continue;
      if (na == 0.0) {
        for (int q = 0; q < 6; ++q) out.d[q] = b[2 + q];
      } else {
        comoments_merge(na, out.d, b[0], b + 2);
      }
      na += b[0];
    }
  }
}

__global__ void xchg_pack_kernel(const Acc* acc, const uint8_t* hll, const int32_t* kinds, int T,
                                 int nh, int64_t rows, int64_t* isum, int64_t* imax, double* mom,
                                 uint8_t* hll_out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < T) xchg_pack_task(kinds[i], acc[i], i, T, isum, imax, mom);
  if (i < nh) hll_out[i] = hll[i];
  if (i == 0) isum[10 * T] = rows;
}

__global__ void xchg_unpack_kernel(const int32_t* kinds, int T, int nh, int world,
                                   const int64_t* isum, const int64_t* imax, const double* momg,
                                   const uint8_t* hll_in, Acc* acc, uint8_t* hll, int64_t* rows) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < T) xchg_merge_task(kinds[i], i, T, world, isum, imax, momg, acc[i]);
  if (i < nh) hll[i] = hll_in[i];
  if (i == 0) *rows = isum[10 * T];
}

// The plan's task kinds on the device, uploaded once per state (stream-ordered before the first
// exchange kernel that reads them; the host vector lives in the state until then).
dq_status xchg_kinds(dq_state* s, hipStream_t st) {
  if (s->kinds_ready) return DQ_OK;
  const dq_plan* p = s->plan;
  s->h_kinds.assign(std::max<size_t>(1, p->tasks.size()), 0);
  for (size_t t = 0; t < p->tasks.size(); ++t) s->h_kinds[t] = p->tasks[t].kind;
  HIP_TRY(s->d_kinds.ensure(s->h_kinds.size()));
  HIP_TRY(hipMemcpyAsync(s->d_kinds.p, s->h_kinds.data(), s->h_kinds.size() * 4,
                         hipMemcpyHostToDevice, st));
  s->kinds_ready = true;
  return DQ_OK;
}
}  // namespace

extern "C" dq_status dq_state_exchange_sizes(const dq_plan* plan, int64_t* n_sum, int64_t* n_max,
                                             int64_t* n_mom, int64_t* n_hll) {
  if (!plan || !n_sum || !n_max || !n_mom || !n_hll)
    return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  const int64_t T = (int64_t)plan->tasks.size();
  *n_sum = 10 * T + 1;
  *n_max = 2 * T;
  *n_mom = kMomW * T;
  *n_hll = (int64_t)plan->n_hll * kHllM;
  return DQ_OK;
}

extern "C" dq_status dq_state_exchange_pack(dq_state* s, int64_t* isum, int64_t* imax, double* mom,
                                            uint8_t* hll, void* hip_stream) {
  if (!s || !isum || !imax || !mom || (!hll && s->plan->n_hll))
    return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  const dq_plan* p = s->plan;
  const int T = (int)p->tasks.size(), nh = (int)s->hll.size();
  if (s->device < 0) {  // host-only state: host buffers
    for (int k = 0; k < T; ++k) xchg_pack_task(p->tasks[k].kind, s->acc[k], k, T, isum, imax, mom);
    for (int i = 0; i < nh; ++i) hll[i] = s->hll[i];
    isum[10 * (size_t)T] = s->rows;
    return DQ_OK;
  }
  if (s->rows_on_device)
    return fail(DQ_ERR_STATE, "state holds an unsynced exchange result (call dq_state_sync)");
  HIP_TRY(hipSetDevice(s->device));
  hipStream_t cs = reinterpret_cast<hipStream_t>(hip_stream);
  hipStream_t st = s->stream_set ? s->stream : cs;
  // the host mirror is newer than the device words (a merge / deserialize): upload it first, on
  // the state's stream
  if (!s->stream_set) {
    s->stream = st;
    s->stream_set = true;
  }
  dq_status us = upload_host(s);
  if (us != DQ_OK) return us;
  if (s->reset_pending) {  // reset and never scanned: the device words are stale, pack the mirror
    s->host_dirty = true;
    us = upload_host(s);
    if (us != DQ_OK) return us;
  }
  dq_status ks = xchg_kinds(s, st);
  if (ks != DQ_OK) return ks;
  const int n = std::max(std::max(T, nh), 1);
  hipLaunchKernelGGL(xchg_pack_kernel, dim3((n + 255) / 256), dim3(256), 0, st, s->d_acc.p, s->d_hll.p,
                     s->d_kinds.p, T, nh, s->rows, isum, imax, mom, hll);
  HIP_TRY(hipGetLastError());
  if (cs != st) {  // order the caller's stream (the collectives) after the pack
    HIP_TRY(hipEventRecord(s->ev_xchg, st));
    HIP_TRY(hipStreamWaitEvent(cs, s->ev_xchg, 0));
  }
  return DQ_OK;
}

extern "C" dq_status dq_state_exchange_unpack(dq_state* s, const int64_t* isum, const int64_t* imax,
                                              const double* mom_gathered, const uint8_t* hll,
                                              int world, void* hip_stream) {
  if (!s || !isum || !imax || (!mom_gathered && !s->plan->tasks.empty()) ||
      (!hll && s->plan->n_hll) || world < 1)
    return fail(DQ_ERR_INVALID_ARGUMENT, "bad argument");
  const dq_plan* p = s->plan;
  const int T = (int)p->tasks.size(), nh = (int)s->hll.size();
  if (s->device < 0) {
    for (int k = 0; k < T; ++k) xchg_merge_task(p->tasks[k].kind, k, T, world, isum, imax, mom_gathered, s->acc[k]);
    for (int i = 0; i < nh; ++i) s->hll[i] = hll[i];
    s->rows = isum[10 * (size_t)T];
    s->synced = true;
    s->host_dirty = true;
    return DQ_OK;
  }
  HIP_TRY(hipSetDevice(s->device));
  hipStream_t cs = reinterpret_cast<hipStream_t>(hip_stream);
  if (!s->stream_set) {
    s->stream = cs;
    s->stream_set = true;
  }
  hipStream_t st = s->stream;
  if (cs != st) {
    HIP_TRY(hipEventRecord(s->ev_xchg, cs));
    HIP_TRY(hipStreamWaitEvent(st, s->ev_xchg, 0));
  }
  dq_status ks = xchg_kinds(s, st);
  if (ks != DQ_OK) return ks;
  HIP_TRY(s->d_rows.ensure(1));
  const int n = std::max(std::max(T, nh), 1);
  hipLaunchKernelGGL(xchg_unpack_kernel, dim3((n + 255) / 256), dim3(256), 0, st, s->d_kinds.p, T, nh,
                     world, isum, imax, mom_gathered, hll, s->d_acc.p, s->d_hll.p, s->d_rows.p);
  HIP_TRY(hipGetLastError());
  s->rows_on_device = true;
  s->synced = false;
  s->host_dirty = false;
  s->reset_pending = false;
  return DQ_OK;
}

extern "C" dq_status dq_state_merge(dq_state* dst, const dq_state* src) {
  if (!dst || !src) return fail(DQ_ERR_INVALID_ARGUMENT, "null state");
  if (dst->plan != src->plan) return fail(DQ_ERR_STATE, "states belong to different plans");
  if (!dst->synced || !src->synced) return fail(DQ_ERR_STATE, "states must be synced before merging");
  const dq_plan* p = dst->plan;
  for (size_t k = 0; k < p->tasks.size(); ++k) acc_merge(p->tasks[k].kind, dst->acc[k], src->acc[k]);
  for (size_t k = 0; k < dst->hll.size(); ++k) dst->hll[k] = std::max(dst->hll[k], src->hll[k]);
  dst->rows += src->rows;
  dst->host_dirty = true;
  return DQ_OK;
}

static const uint64_t kMagic = 0x3130514445455144ULL;  // "DQEEDQ01"

extern "C" int64_t dq_state_serialized_size(const dq_plan* plan) {
  if (!plan) return -1;
  return 32 + (int64_t)plan->tasks.size() * (int64_t)sizeof(Acc) + (int64_t)plan->n_hll * kHllM;
}

extern "C" dq_status dq_state_serialize(const dq_state* s, void* buf, int64_t buf_len) {
  if (!s || !buf) return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  if (!s->synced) return fail(DQ_ERR_STATE, "state not synced");
  int64_t need = dq_state_serialized_size(s->plan);
  if (buf_len < need) return fail(DQ_ERR_INVALID_ARGUMENT, "buffer too small (%lld < %lld)",
                                  (long long)buf_len, (long long)need);
  uint8_t* b = static_cast<uint8_t*>(buf);
  uint64_t hdr[4] = {kMagic, (uint64_t)s->plan->tasks.size(), (uint64_t)s->plan->n_hll, (uint64_t)s->rows};
  memcpy(b, hdr, 32);
  if (!s->acc.empty()) memcpy(b + 32, s->acc.data(), s->acc.size() * sizeof(Acc));
  if (!s->hll.empty()) memcpy(b + 32 + s->acc.size() * sizeof(Acc), s->hll.data(), s->hll.size());
  return DQ_OK;
}

extern "C" dq_status dq_state_deserialize(dq_state* s, const void* buf, int64_t buf_len) {
  if (!s || !buf) return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  int64_t need = dq_state_serialized_size(s->plan);
  if (buf_len < need) return fail(DQ_ERR_INVALID_ARGUMENT, "buffer too small");
  const uint8_t* b = static_cast<const uint8_t*>(buf);
  uint64_t hdr[4];
  memcpy(hdr, b, 32);
  if (hdr[0] != kMagic || hdr[1] != s->plan->tasks.size() || hdr[2] != (uint64_t)s->plan->n_hll)
    return fail(DQ_ERR_STATE, "serialized state does not match this plan");
  if (s->stream_set && s->device >= 0) HIP_TRY(host_wait(s->stream));
  s->rows = (int64_t)hdr[3];
  if (!s->acc.empty()) memcpy(s->acc.data(), b + 32, s->acc.size() * sizeof(Acc));
  if (!s->hll.empty()) memcpy(s->hll.data(), b + 32 + s->acc.size() * sizeof(Acc), s->hll.size());
  s->synced = true;
  s->host_dirty = true;
  return DQ_OK;
}

// ------------------------------------------------------------------------------------------------
// HLL estimate and hash (host)
// ------------------------------------------------------------------------------------------------
extern "C" double dq_hll_count(const uint64_t* words, int* bias_corrected) {
  // HyperLogLogPlusPlusUtils.count (StatefulHyperloglogPlus.scala:208-255)
  const double M = kHllM;
  const double alpha_m2 = (0.7213 / (1.0 + 1.079 / M)) * M * M;
  double z_inv = 0.0, V = 0.0;
  int idx = 0;
  for (int w = 0; w < kHllWords; ++w) {
    uint64_t word = words[w];
    for (int i = 0; i < kHllRegsPerWord && idx < kHllM; ++i, ++idx) {
      uint64_t m = (word >> (kHllRegBits * i)) & 0x3f;
      // `1.0 / (1 << Midx)` (:220): `1` is a Scala Int and Midx a Long, so the JVM shifts a 32-bit
      // int by Midx & 31 (JLS 15.19): register 31 adds 1/Int.MinValue = -2^-31 and a register
      // m >= 32 adds 2^-(m-32).  Restated literally -- the estimate must equal deequ's.
      z_inv += 1.0 / (double)(int32_t)(1u << (m & 31));
      if (m == 0) V += 1.0;
    }
  }
  const double threshold = 400.0;  // HyperLogLogPlusPlus.THRESHOLDS(P - 4), P = 9
  double e = alpha_m2 / z_inv;
  bool biased = e < 5.0 * M;
  double estimate;
  if (V > 0) {
    double H = M * std::log(M / V);
    if (H <= threshold) {
      estimate = H;
      biased = false;
    } else {
      estimate = e;
    }
  } else {
    estimate = e;
  }
  if (bias_corrected) *bias_corrected = biased ? 1 : 0;
  // JDK 8 Math.round(double): (long) floor(a + 0.5) except for the largest double below 0.5; the
  // (long) cast saturates and maps NaN to 0 (JLS 5.1.3).  A register >= 31 can make zInverse
  // tiny or negative, so the saturating cases are reachable.
  if (estimate != estimate || estimate == 0x1.fffffffffffffp-2) return 0.0;
  const double f = std::floor(estimate + 0.5);
  if (f >= 9223372036854775808.0) return (double)INT64_MAX;
  if (f <= -9223372036854775808.0) return (double)INT64_MIN;
  return (double)(int64_t)f;
}

extern "C" uint64_t dq_xxhash64(const void* data, int64_t nbytes, uint64_t seed) {
  HostBytes rd{static_cast<const uint8_t*>(data)};
  return xxh_bytes(rd, nbytes, seed);
}

extern "C" int dq_java_double_to_string(double value, char* buf) {
  return jfmt::double_to_java(value, buf);
}
extern "C" int dq_java_float_to_string(float value, char* buf) {
  return jfmt::float_to_java(value, buf);
}
extern "C" void dq_java_doubles_to_strings(const double* values, int64_t n, int is_float, char* out,
                                           int32_t* lens) {
  for (int64_t i = 0; i < n; ++i)
    lens[i] = is_float ? jfmt::float_to_java((float)values[i], out + 32 * i)
                       : jfmt::double_to_java(values[i], out + 32 * i);
}

extern "C" double dq_decimal_to_double(uint64_t lo, int64_t hi, int32_t scale) {
  return dec_to_double(lo, hi, scale < 0 ? 0 : (scale > 38 ? 38 : scale));
}

extern "C" dq_status dq_format_values(int32_t type, const void* values, int64_t n, char* out,
                                      int32_t* lens) {
  if (n < 0 || (n > 0 && (!values || !out || !lens))) return fail(DQ_ERR_INVALID_ARGUMENT, "bad argument");
  if (!valid_type(type)) return fail(DQ_ERR_INVALID_ARGUMENT, "unknown column type %d", type);
  for (int64_t i = 0; i < n; ++i) {
    char* o = out + (int64_t)kFmtMax * i;
    if (is_decimal(type)) {
      const uint64_t* v = static_cast<const uint64_t*>(values) + 2 * i;
      lens[i] = dec_format(v[0], (int64_t)v[1], DQ_DECIMAL_SCALE(type), o);
    } else if (type == DQ_DATE32) {
      lens[i] = date_format(static_cast<const int32_t*>(values)[i], o);
    } else if (type == DQ_TIMESTAMP_US) {
      lens[i] = ts_format(static_cast<const int64_t*>(values)[i], o);
    } else {
      return fail(DQ_ERR_WRONG_TYPE, "dq_format_values formats decimal / date / timestamp values");
    }
  }
  return DQ_OK;
}

// Bitmaps re-based for sliced Arrow arrays, owned by the library until dq_column_release.
namespace {
struct OwnedBitmap {
  int device;  // -1: host malloc
  size_t bytes;
};
std::mutex& owned_mutex() {
  static std::mutex m;
  return m;
}
std::map<const void*, OwnedBitmap>& owned_bitmaps() {
  static auto* m = new std::map<const void*, OwnedBitmap>;
  return *m;
}

// A bitmap of `rows` bits starting at bit `bit` of `src`, as a pointer to bit 0: aliases src when
// the offset is whole bytes, else a re-based copy in src's memory space (device or host).
dq_status bitmap_at(const uint8_t* src, int64_t bit, int64_t rows, const uint8_t** out) {
  if (bit % 8 == 0 || rows == 0) {
    *out = src + bit / 8;
    return DQ_OK;
  }
  hipPointerAttribute_t attr{};
  const bool on_device = hipPointerGetAttributes(&attr, src) == hipSuccess &&
                         attr.type == hipMemoryTypeDevice;
  (void)hipGetLastError();  // an unregistered host pointer leaves an error behind
  const size_t n = (size_t)(rows + 7) / 8;
  if (on_device) {
    int cur = 0;
    HIP_TRY(hipGetDevice(&cur));
    HIP_TRY(hipSetDevice(attr.device));
    void* p = nullptr;
    size_t got = 0;
    int dev = 0;
    hipError_t e = dev_alloc(&p, n + 16, &got, &dev);
    if (e == hipSuccess) e = hipMemsetAsync(p, 0, got, nullptr);
    if (e == hipSuccess) e = launch_bitmap_rebase(src, bit, rows, static_cast<uint8_t*>(p), nullptr);
    if (e == hipSuccess) e = host_wait(nullptr);
    (void)hipSetDevice(cur);
    if (e != hipSuccess) {
      if (p) dev_free(p, got, dev);
      return fail(e == hipErrorOutOfMemory ? DQ_ERR_OUT_OF_MEMORY : DQ_ERR_DEVICE,
                  "re-basing a sliced bitmap: %s", hipGetErrorString(e));
    }
    std::lock_guard<std::mutex> lock(owned_mutex());
    owned_bitmaps()[p] = OwnedBitmap{dev, got};
    *out = static_cast<const uint8_t*>(p);
    return DQ_OK;
  }
  auto* h = static_cast<uint8_t*>(std::calloc(n + 16, 1));
  if (!h) return fail(DQ_ERR_OUT_OF_MEMORY, "re-basing a sliced bitmap");
  const int64_t last = (bit + rows - 1) / 8;
  const unsigned sh = (unsigned)(bit & 7);
  for (size_t i = 0; i < n; ++i) {
    const int64_t j = bit / 8 + (int64_t)i;
    unsigned v = src[j] >> sh;
    if (j + 1 <= last) v |= (unsigned)src[j + 1] << (8 - sh);
    h[i] = (uint8_t)v;
  }
  std::lock_guard<std::mutex> lock(owned_mutex());
  owned_bitmaps()[h] = OwnedBitmap{-1, n + 16};
  *out = h;
  return DQ_OK;
}

void release_owned(const void* p) {
  if (!p) return;
  OwnedBitmap b{};
  {
    std::lock_guard<std::mutex> lock(owned_mutex());
    auto it = owned_bitmaps().find(p);
    if (it == owned_bitmaps().end()) return;
    b = it->second;
    owned_bitmaps().erase(it);
  }
  if (b.device < 0) std::free(const_cast<void*>(p));
  else dev_free(const_cast<void*>(p), b.bytes, b.device);
}
}  // namespace

extern "C" dq_status dq_column_from_arrow(const struct ArrowArray* array,
                                          const struct ArrowSchema* schema, dq_column* out) {
  if (!array || !schema || !out || !schema->format)
    return fail(DQ_ERR_INVALID_ARGUMENT, "null argument");
  if (array->offset < 0 || array->length < 0)
    return fail(DQ_ERR_INVALID_ARGUMENT, "negative Arrow offset or length");
  std::string f(schema->format);
  int type = 0;
  if (f == "b") type = DQ_BOOL;
  else if (f == "c") type = DQ_INT8;
  else if (f == "s") type = DQ_INT16;
  else if (f == "i") type = DQ_INT32;
  else if (f == "l") type = DQ_INT64;
  else if (f == "f") type = DQ_FLOAT32;
  else if (f == "g") type = DQ_FLOAT64;
  else if (f == "u") type = DQ_UTF8;
  else if (f == "tdD") type = DQ_DATE32;
  else if (f.compare(0, 4, "tsu:") == 0) type = DQ_TIMESTAMP_US;  // any zone: the values are UTC
  else if (f.compare(0, 2, "d:") == 0) {  // "d:precision,scale[,bitwidth]"
    int prec = -1, sc = -1, bw = 128;
    char tail = 0;
    const int got = sscanf(f.c_str() + 2, "%d,%d,%d%c", &prec, &sc, &bw, &tail);
    if (got < 2 || got > 3 || bw != 128 || prec < 1 || prec > 38 || sc < 0 || sc > prec)
      return fail(DQ_ERR_UNSUPPORTED, "Arrow decimal format '%s' (decimal128, 1 <= p <= 38, "
                                      "0 <= s <= p)", schema->format);
    type = DQ_DECIMAL_TYPE(prec, sc);
  } else return fail(DQ_ERR_UNSUPPORTED, "Arrow format '%s'", schema->format);
  int64_t need = type == DQ_UTF8 ? 3 : 2;
  if (array->n_buffers < need) return fail(DQ_ERR_INVALID_ARGUMENT, "too few Arrow buffers");
  const int64_t off = array->offset, n = array->length;
  dq_column c{};
  c.type = type;
  c.data_bytes = 0;  // unknown: the Arrow C Data Interface carries no buffer sizes
  c.length = n;
  const auto* valid = static_cast<const uint8_t*>(array->buffers[0]);
  if (array->null_count != 0 && valid) {
    dq_status st = bitmap_at(valid, off, n, &c.validity);
    if (st != DQ_OK) return st;
  }
  const auto* vals = static_cast<const uint8_t*>(array->buffers[1]);
  if (type == DQ_BOOL) {
    const uint8_t* v = nullptr;
    dq_status st = vals ? bitmap_at(vals, off, n, &v) : DQ_OK;
    if (st != DQ_OK) {
      release_owned(c.validity);
      return st;
    }
    c.values = v;
  } else if (type == DQ_UTF8) {  // offsets stay absolute into the (unsliced) character buffer
    c.values = vals ? vals + 4 * off : nullptr;
    c.data = static_cast<const uint8_t*>(array->buffers[2]);
  } else {
    const int64_t w = type_size(type);
    c.values = vals ? vals + w * off : nullptr;
  }
  *out = c;
  return DQ_OK;
}

extern "C" void dq_column_release(dq_column* col) {
  if (!col) return;
  release_owned(col->validity);
  if (col->type == DQ_BOOL) release_owned(col->values);
}

// ------------------------------------------------------------------------------------------------
// Device memory cache (kernels.h)
// ------------------------------------------------------------------------------------------------
#include <chrono>
#include <mutex>

namespace dq {
namespace {
constexpr int kPoolDevices = 64;
constexpr size_t kPoolRound = 256;                 // small blocks: 256-B granules
constexpr size_t kPoolBig = 2ULL << 20;            // >= 2 MiB: 2-MiB granules
// At most a third of the device's memory is cached (96 GB of an MI355X's 288).  Measured on
// configs[4]: with a 32 GB cap the larger freed blocks went back to the driver,
// hipFree of 4-8 GB took 0.1-0.3 s, and about one hipMalloc of such a size in twenty waited
// ~6 s (the driver clearing freed memory); with 96 GB every block is reused.
size_t pool_keep(int dev) {  // the caller holds the pool lock; DQ_POOL_KEEP_GB overrides
  static const long long env_gb = [] {
    const char* e = getenv("DQ_POOL_KEEP_GB");
    return e ? atoll(e) : -1LL;
  }();
  if (env_gb >= 0) return (size_t)env_gb << 30;
  static size_t keep[kPoolDevices] = {0};
  if (!keep[dev]) {
    size_t free_b = 0, total_b = 0;
    keep[dev] = hipMemGetInfo(&free_b, &total_b) == hipSuccess && total_b ? total_b / 3
                                                                           : (32ULL << 30);
  }
  return keep[dev];
}
int pool_debug() {  // DQ_POOL_DEBUG=1: every hipMalloc / hipFree of the cache taking >= 50 ms
  static const int d = [] {
    const char* e = getenv("DQ_POOL_DEBUG");
    return e ? atoi(e) : 0;
  }();
  return d;
}
double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}
struct DevPool {
  std::mutex m;
  std::multimap<size_t, void*> free_blocks[kPoolDevices];
  size_t cached[kPoolDevices] = {0};
};
DevPool& dev_pool() {
  static DevPool* pool = new DevPool;  // lives to process exit (the driver reclaims the memory)
  return *pool;
}
size_t pool_round(size_t b) {
  const size_t g = b >= kPoolBig ? kPoolBig : kPoolRound;
  return (b + g - 1) / g * g;
}
void release_cached(int dev) {  // caller holds the lock; dev is the current device
  DevPool& pool = dev_pool();
  for (auto& kv : pool.free_blocks[dev]) (void)hipFree(kv.second);
  pool.free_blocks[dev].clear();
  pool.cached[dev] = 0;
}
}  // namespace

hipError_t dev_alloc(void** out, size_t bytes, size_t* got, int* device) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  *device = dev;
  const size_t want = pool_round(bytes ? bytes : 1);
  DevPool& pool = dev_pool();
  if (dev >= 0 && dev < kPoolDevices) {
    std::lock_guard<std::mutex> lock(pool.m);
    auto& fl = pool.free_blocks[dev];
    auto it = fl.lower_bound(want);
    if (it != fl.end() && it->first <= 2 * want) {
      *out = it->second;
      *got = it->first;
      pool.cached[dev] -= it->first;
      fl.erase(it);
      return hipSuccess;
    }
  }
  auto t0 = std::chrono::steady_clock::now();
  hipError_t e = hipMalloc(out, want);
  if (pool_debug() && ms_since(t0) >= 50.0)
    fprintf(stderr, "dq pool: hipMalloc(%.2f GB) took %.1f ms (cached %.2f GB)\n", want / 1e9,
            ms_since(t0), pool.cached[dev] / 1e9);
  if (e == hipErrorOutOfMemory && dev >= 0 && dev < kPoolDevices) {
    (void)hipGetLastError();
    {
      std::lock_guard<std::mutex> lock(pool.m);
      release_cached(dev);
    }
    e = hipMalloc(out, want);
  }
  *got = e == hipSuccess ? want : 0;
  return e;
}

void dev_free(void* p, size_t bytes, int dev) {
  if (!p) return;
  int cur = 0;
  (void)hipGetDevice(&cur);
  if (dev != cur) (void)hipSetDevice(dev);
  (void)hipDeviceSynchronize();  // as hipFree: no kernel may still use the block
  DevPool& pool = dev_pool();
  bool kept = false;
  if (dev >= 0 && dev < kPoolDevices && bytes) {
    std::lock_guard<std::mutex> lock(pool.m);
    if (pool.cached[dev] + bytes <= pool_keep(dev)) {
      pool.free_blocks[dev].emplace(bytes, p);
      pool.cached[dev] += bytes;
      kept = true;
    }
  }
  if (!kept) {
    auto t0 = std::chrono::steady_clock::now();
    (void)hipFree(p);
    if (pool_debug() && ms_since(t0) >= 50.0)
      fprintf(stderr, "dq pool: hipFree(%.2f GB) took %.1f ms\n", bytes / 1e9, ms_since(t0));
  }
  if (dev != cur) (void)hipSetDevice(cur);
}

namespace {
struct PinnedPool {  // page-locked staging blocks (powers of two >= 4 KB), at most kPinnedKeep
  std::mutex m;
  std::multimap<size_t, void*> free_blocks;
  size_t cached = 0;
};
constexpr size_t kPinnedKeep = 256u << 20;  // bytes of idle blocks kept for reuse
PinnedPool& pinned_pool() {
  static PinnedPool* pool = new PinnedPool;
  return *pool;
}
}  // namespace

void release_pinned_staging() {
  PinnedPool& pool = pinned_pool();
  std::lock_guard<std::mutex> lock(pool.m);
  for (auto& kv : pool.free_blocks) (void)hipHostFree(kv.second);
  pool.free_blocks.clear();
  pool.cached = 0;
}

hipError_t d2h(void* dst, const void* src, size_t bytes, hipStream_t st) {
  const D2HPart part{dst, src, bytes};
  return d2h_n(&part, 1, st);
}

hipError_t d2h_n(const D2HPart* parts, int n, hipStream_t st) {
  size_t total = 0;
  for (int i = 0; i < n; ++i) total += (parts[i].bytes + 15) & ~(size_t)15;
  if (!total) return host_wait(st);
  size_t want = 4096;
  while (want < total) want <<= 1;
  PinnedPool& pool = pinned_pool();
  void* buf = nullptr;
  {
    std::lock_guard<std::mutex> lock(pool.m);
    auto it = pool.free_blocks.lower_bound(want);
    if (it != pool.free_blocks.end()) {
      want = it->first;
      buf = it->second;
      pool.cached -= want;
      pool.free_blocks.erase(it);
    }
  }
  if (!buf && want > (64u << 20)) {  // (large copies: not worth pinning a block for)
    hipError_t e = host_wait(st);
    for (int i = 0; i < n && e == hipSuccess; ++i)
      if (parts[i].bytes) e = hipMemcpy(parts[i].dst, parts[i].src, parts[i].bytes, hipMemcpyDeviceToHost);
    return e;
  }
  if (!buf) {
    hipError_t e = hipHostMalloc(&buf, want, hipHostMallocDefault);
    if (e != hipSuccess) return e;
  }
  hipError_t e = hipSuccess;
  size_t off = 0;
  for (int i = 0; i < n && e == hipSuccess; ++i) {
    if (parts[i].bytes)
      e = hipMemcpyAsync(static_cast<char*>(buf) + off, parts[i].src, parts[i].bytes, hipMemcpyDeviceToHost, st);
    off += (parts[i].bytes + 15) & ~(size_t)15;
  }
  if (e == hipSuccess) e = host_wait(st);
  if (e != hipSuccess) return e;  // (the block is dropped: a DMA may still be writing it)
  off = 0;
  for (int i = 0; i < n; ++i) {
    if (parts[i].bytes) memcpy(parts[i].dst, static_cast<char*>(buf) + off, parts[i].bytes);
    off += (parts[i].bytes + 15) & ~(size_t)15;
  }
  bool keep;
  {
    std::lock_guard<std::mutex> lock(pool.m);
    keep = pool.cached + want <= kPinnedKeep;
    if (keep) {
      pool.free_blocks.emplace(want, buf);
      pool.cached += want;
    }
  }
  if (!keep) (void)hipHostFree(buf);
  return hipSuccess;
}

}  // namespace dq

extern "C" int64_t dq_cached_device_bytes(int device) {
  if (device < 0 || device >= dq::kPoolDevices) return 0;
  dq::DevPool& pool = dq::dev_pool();
  std::lock_guard<std::mutex> lock(pool.m);
  return (int64_t)pool.cached[device];
}

extern "C" void dq_release_cached_memory(void) {
  int cur = 0;
  (void)hipGetDevice(&cur);
  int n = 0;
  (void)hipGetDeviceCount(&n);
  dq::DevPool& pool = dq::dev_pool();
  std::lock_guard<std::mutex> lock(pool.m);
  for (int d = 0; d < n && d < dq::kPoolDevices; ++d) {
    if (pool.free_blocks[d].empty()) continue;
    (void)hipSetDevice(d);
    dq::release_cached(d);
  }
  (void)hipSetDevice(cur);
  dq::release_pinned_staging();
}
