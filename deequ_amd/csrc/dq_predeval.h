// dq_predeval.h -- the predicate IR's semantics, one source for the device interpreter
// (dq_pred.hip: dq_pred_kernel evaluates every non-inline Compliance predicate and `where` filter)
// and its host build (dq_api.cpp: dq_diag_eval_predicate, which CPU tests check against the
// oracle's independent SQL evaluator).  Internal, not ABI.
//
// Spark parses each predicate with `expr(String)` (Compliance.scala:49, Analyzer.scala:409-432);
// its analyzer makes every coercion an explicit Cast node (Spark 2.2.2 TypeCoercion), which the
// encoder turns into DQ_P_CAST / DQ_P_CAST_DOUBLE.  Cast semantics restated here (Spark 2.2.2
// Cast.castToByte/Short/Int/Long/Float/Double/Boolean, non-ANSI):
//   integral -> narrower integral : keep the low bits (Scala .toInt / .toShort / .toByte);
//   fractional -> int / long       : Java d2i / d2l (NaN -> 0, saturating, toward zero);
//   fractional -> short / byte     : d2i, then keep the low bits (`numeric.toInt(b).toShort`);
//   integral -> float              : Java l2f, correctly rounded from the integer itself;
//   double -> float                : IEEE round to nearest even (Infinity past Float.MAX_VALUE);
//   boolean -> numeric             : 1 / 0;  numeric -> boolean: value != 0 (NaN -> true).
// A float value travels as the fp64 holding it exactly, so comparisons in fp64 order float
// values as FloatType does.
#pragma once

#include "dq_internal.h"
#include "dq_numparse.h"

namespace dq {
namespace pred {

enum ValType : uint8_t { VT_INT = 0, VT_FLT = 1, VT_BOOL = 2, VT_STR = 3 };

struct Val {
  int64_t i;      // int / bool value; string length for VT_STR
  double f;
  uint8_t type;
  uint8_t null;
  const uint8_t* s;  // VT_STR bytes
};

struct Bytes {  // byte source of dq_numparse.h over a plain pointer
  const uint8_t* p;
  DQ_HD uint32_t operator[](int32_t i) const { return p[i]; }
};

DQ_HD inline Val make(int64_t i, double f, uint8_t type, uint8_t null) {
  Val v;
  v.i = i;
  v.f = f;
  v.type = type;
  v.null = null;
  v.s = nullptr;
  return v;
}

// UTF8String.compareTo: unsigned byte-wise, then shorter first.
DQ_HD inline int ord_str(const Val& a, const Val& b) {
  const int64_t n = a.i < b.i ? a.i : b.i;
  for (int64_t k = 0; k < n; ++k) {
    const int d = (int)a.s[k] - (int)b.s[k];
    if (d) return d < 0 ? -1 : 1;
  }
  return (int)(a.i > b.i) - (int)(a.i < b.i);
}

DQ_HD inline bool col_valid(const DevColumn& c, int64_t row) {
  return c.validity == nullptr || ((c.validity[row >> 3] >> (row & 7)) & 1u);
}

DQ_HD inline Val load_col(const DevColumn& c, int64_t row) {
  Val v = make(0, 0.0, VT_INT, col_valid(c, row) ? 0 : 1);
  switch (c.type) {
    case DQ_T_UTF8: {
      const int32_t b = c.offsets[row], e = c.offsets[row + 1];
      v.s = static_cast<const uint8_t*>(c.values) + b;
      v.i = e - b;
      v.type = VT_STR;
      break;
    }
    case DQ_T_BOOL: {
      const uint8_t* b = static_cast<const uint8_t*>(c.values);
      v.i = (b[row >> 3] >> (row & 7)) & 1u;
      v.type = VT_BOOL;
      break;
    }
    case DQ_T_INT8: v.i = static_cast<const int8_t*>(c.values)[row]; break;
    case DQ_T_INT16: v.i = static_cast<const int16_t*>(c.values)[row]; break;
    case DQ_T_INT32: v.i = static_cast<const int32_t*>(c.values)[row]; break;
    case DQ_T_INT64: v.i = static_cast<const int64_t*>(c.values)[row]; break;
    case DQ_T_FLOAT32: v.f = static_cast<const float*>(c.values)[row]; v.type = VT_FLT; break;
    case DQ_T_FLOAT64: v.f = static_cast<const double*>(c.values)[row]; v.type = VT_FLT; break;
    default: v.null = 1; break;
  }
  return v;
}

DQ_HD inline double as_f64(const Val& v) { return v.type == VT_FLT ? v.f : (double)v.i; }

// Spark's NaN-safe double ordering: NaN equals NaN and is larger than every other value.
DQ_HD inline int ord_f64(double a, double b) {
  const bool an = a != a, bn = b != b;
  if (an | bn) return (int)an - (int)bn;
  return (int)(a > b) - (int)(a < b);
}

DQ_HD inline bool cmp_result(int opcode, int ord) {
  switch (opcode) {
    case DQ_P_EQ: return ord == 0;
    case DQ_P_NE: return ord != 0;
    case DQ_P_LT: return ord < 0;
    case DQ_P_LE: return ord <= 0;
    case DQ_P_GT: return ord > 0;
    case DQ_P_GE: return ord >= 0;
    default: return ord == 0;
  }
}

// Java d2l / d2i: NaN -> 0, out-of-range saturates, otherwise truncation toward zero.
DQ_HD inline int64_t java_d2l(double d) {
  if (d != d) return 0;
  if (d >= 9223372036854775808.0) return INT64_MAX;
  if (d <= -9223372036854775808.0) return INT64_MIN;
  return (int64_t)d;
}
DQ_HD inline int64_t java_d2i(double d) {
  if (d != d) return 0;
  if (d >= 2147483647.0) return INT32_MAX;
  if (d <= -2147483648.0) return INT32_MIN;
  return (int64_t)(int32_t)d;
}

// DQ_P_CAST of a non-string value to `target` (a dq_type); the validator has rejected every
// other combination.  A NULL stays NULL (its payload is irrelevant).
DQ_HD inline void cast_value(Val& a, int target) {
  const bool flt = a.type == VT_FLT;
  switch (target) {
    case DQ_T_INT64: a.i = flt ? java_d2l(a.f) : a.i; a.type = VT_INT; break;
    case DQ_T_INT32: a.i = (int64_t)(int32_t)(uint32_t)(uint64_t)(flt ? java_d2i(a.f) : a.i); a.type = VT_INT; break;
    case DQ_T_INT16: a.i = (int64_t)(int16_t)(uint16_t)(uint64_t)(flt ? java_d2i(a.f) : a.i); a.type = VT_INT; break;
    case DQ_T_INT8: a.i = (int64_t)(int8_t)(uint8_t)(uint64_t)(flt ? java_d2i(a.f) : a.i); a.type = VT_INT; break;
    case DQ_T_FLOAT32: a.f = flt ? (double)(float)a.f : (double)(float)a.i; a.type = VT_FLT; break;
    case DQ_T_FLOAT64: a.f = as_f64(a); a.type = VT_FLT; break;
    case DQ_T_BOOL: a.i = flt ? (a.f != 0.0 ? 1 : 0) : (a.i != 0 ? 1 : 0); a.type = VT_BOOL; break;
    default: a.null = 1; break;
  }
}

// One row of a validated program.  CAST: the program casts a string to double
// (Double.parseDouble, whose exact slow path carries ~1 KB of private scratch per lane on the
// device); programs without one are compiled without the parser.
template <bool CAST>
DQ_HD inline void eval_program(const PredInsn* code, int n, const uint8_t* pool, const DevColumn* cols,
                               int64_t row, bool& t, bool& nn) {
  Val st[kMaxStack];
  int sp = 0;
  for (int pc = 0; pc < n; ++pc) {
    const PredInsn ins = code[pc];
    switch (ins.opcode) {
      case DQ_P_COLUMN: st[sp++] = load_col(cols[ins.arg], row); break;
      case DQ_P_LIT_INT: st[sp++] = make(ins.i64, 0.0, VT_INT, 0); break;
      case DQ_P_LIT_FLOAT: st[sp++] = make(0, ins.f64, VT_FLT, 0); break;
      case DQ_P_LIT_NULL: st[sp++] = make(0, 0.0, VT_INT, 1); break;
      case DQ_P_LIT_STRING: {
        Val v = make((int64_t)ins.arg, 0.0, VT_STR, 0);
        v.s = pool + ins.i64;
        st[sp++] = v;
        break;
      }
      case DQ_P_CAST_DOUBLE: {  // Spark 2.2 Cast(-> DoubleType): parseDouble of a string
        Val& a = st[sp - 1];
        if (CAST && a.type == VT_STR) {
          double v = 0.0;
          int r = 0;
          if constexpr (CAST) r = a.null ? 0 : numparse::parse_double(Bytes{a.s}, (int32_t)a.i, &v);
          a.null = (r == 1) ? a.null : 1;
          a.f = v;
        } else {
          a.f = as_f64(a);
        }
        a.type = VT_FLT;
        break;
      }
      case DQ_P_CAST: cast_value(st[sp - 1], ins.arg); break;
      case DQ_P_TRUE: st[sp++] = make(1, 0.0, VT_BOOL, 0); break;
      case DQ_P_FALSE: st[sp++] = make(0, 0.0, VT_BOOL, 0); break;
      case DQ_P_COALESCE: {
        Val b = st[--sp];
        Val a = st[sp - 1];
        Val r = a.null ? b : a;
        if ((a.type == VT_FLT) != (b.type == VT_FLT)) {  // common type is fp64
          r.f = as_f64(r);
          r.type = VT_FLT;
        }
        st[sp - 1] = r;
        break;
      }
      case DQ_P_EQ: case DQ_P_NE: case DQ_P_LT: case DQ_P_LE: case DQ_P_GT: case DQ_P_GE:
      case DQ_P_EQ_NULLSAFE: {
        Val b = st[--sp];
        Val a = st[sp - 1];
        Val r = make(0, 0.0, VT_BOOL, 0);
        if (a.null || b.null) {
          if (ins.opcode == DQ_P_EQ_NULLSAFE) r.i = (a.null && b.null) ? 1 : 0;
          else r.null = 1;
        } else {
          int ord;
          if (a.type == VT_STR) ord = ord_str(a, b);
          else if (ins.arg == DQ_CMP_AS_FLOAT64) ord = ord_f64(as_f64(a), as_f64(b));
          else ord = (int)(a.i > b.i) - (int)(a.i < b.i);
          r.i = cmp_result(ins.opcode, ord) ? 1 : 0;
        }
        st[sp - 1] = r;
        break;
      }
      case DQ_P_IS_NULL: st[sp - 1] = make(st[sp - 1].null ? 1 : 0, 0.0, VT_BOOL, 0); break;
      case DQ_P_IS_NOT_NULL: st[sp - 1] = make(st[sp - 1].null ? 0 : 1, 0.0, VT_BOOL, 0); break;
      case DQ_P_NOT: {
        Val a = st[sp - 1];
        if (!a.null) a.i = a.i ? 0 : 1;
        st[sp - 1] = a;
        break;
      }
      case DQ_P_AND: case DQ_P_OR: {
        Val b = st[--sp];
        Val a = st[sp - 1];
        Val r = make(0, 0.0, VT_BOOL, 0);
        const bool at = !a.null && a.i, af = !a.null && !a.i;
        const bool bt = !b.null && b.i, bf = !b.null && !b.i;
        if (ins.opcode == DQ_P_AND) {
          if (af || bf) r.i = 0;
          else if (a.null || b.null) r.null = 1;
          else r.i = 1;
        } else {
          if (at || bt) r.i = 1;
          else if (a.null || b.null) r.null = 1;
          else r.i = 0;
        }
        st[sp - 1] = r;
        break;
      }
      default: break;
    }
  }
  const Val top = st[sp - 1];
  nn = !top.null;
  t = nn && top.i != 0;
}

}  // namespace pred
}  // namespace dq
