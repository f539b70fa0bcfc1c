"""SQL predicate -> dq_pred_insn postfix program (the GPU's Compliance / `where` input).

Spark parses every Compliance predicate and `where` filter with `functions.expr(String)`
(Compliance.scala:49, Analyzer.scala:413-432) and its analyzer resolves the types.  This
module plays that role for the subset deequ's Check DSL emits on numeric columns
(Check.scala:594-943): comparisons, IN, BETWEEN, IS [NOT] NULL, COALESCE, AND/OR/NOT, with
Spark 2.2.2's literal typing and coercion:

* `3` is an integer literal, `3.5` a DECIMAL literal, `3.5e2` / `3.5D` a DOUBLE literal;
* long vs decimal compares exactly (DecimalPrecision); here that is rewritten into an exact
  int64 comparison (x > 3.5  ==>  x >= 4;  x = 3.5  ==>  false-or-NULL);
* anything vs double / float column compares in fp64 with Spark's NaN-safe ordering;
* float vs int / long compares in FloatType: the integral side is rounded to float (a literal on
  the host, a column per row through DQ_P_CAST to FLOAT32);
* `CAST(x AS type)` to TINYINT/SMALLINT/INT/BIGINT, FLOAT, DOUBLE or BOOLEAN becomes DQ_P_CAST
  (the library evaluates Spark 2.2's Cast semantics: narrowing wraps, fractional -> integral is
  Java's saturating d2i / d2l); CAST(string AS DOUBLE) is DQ_P_CAST_DOUBLE.

Column names resolve case-insensitively, as Spark 2.2 does by default
(`spark.sql.caseSensitive=false`); two columns equal but for case make a reference ambiguous.

Arithmetic, functions other than COALESCE / CAST, other casts of strings and UDFs raise
UnsupportedPredicate: the reference's JNI shim would leave such an analyzer on Spark
(SURVEY §8(b) "Eligibility").
"""
from __future__ import annotations

import math
from decimal import Decimal, InvalidOperation
from fractions import Fraction
from typing import Dict, List, Tuple

from . import _lib as L

Insn = Tuple[int, int, int, float]  # (opcode, arg, i64, f64)

_INTEGRAL = {"int8", "int16", "int32", "int64"}
_FRACTIONAL = {"float32", "float64"}

# Spark 2.2 SQL type names (SqlBase.g4 primitive types) -> dq_type names the IR casts to
_CAST_TYPES = {"TINYINT": "int8", "BYTE": "int8", "SMALLINT": "int16", "SHORT": "int16",
               "INT": "int32", "INTEGER": "int32", "BIGINT": "int64", "LONG": "int64",
               "FLOAT": "float32", "REAL": "float32", "DOUBLE": "float64", "BOOLEAN": "bool"}


class UnsupportedPredicate(ValueError):
    """The predicate is valid SQL but not in the GPU-eligible subset."""


class PredicateSyntaxError(ValueError):
    pass


# ----------------------------------------------------------------------------- lexer
def _tokenize(text: str):
    toks, i, n = [], 0, len(text)
    while i < n:
        ch = text[i]
        if ch.isspace():
            i += 1
            continue
        if ch == "'" or ch == '"':
            j = i + 1
            buf = []
            while j < n and text[j] != ch:
                if text[j] == "\\" and j + 1 < n:
                    j += 1
                buf.append(text[j])
                j += 1
            if j >= n:
                raise PredicateSyntaxError("unterminated string literal in %r" % text)
            toks.append(("STR", "".join(buf)))
            i = j + 1
            continue
        if ch == "`":
            j = text.find("`", i + 1)
            if j < 0:
                raise PredicateSyntaxError("unterminated identifier in %r" % text)
            toks.append(("ID", text[i + 1:j]))
            i = j + 1
            continue
        if ch.isdigit() or (ch == "." and i + 1 < n and text[i + 1].isdigit()):
            j = i
            while j < n and (text[j].isdigit() or text[j] == "."):
                j += 1
            kind = "DEC" if "." in text[i:j] else "INT"
            if j < n and text[j] in "eE" and j + 1 < n and (text[j + 1].isdigit() or text[j + 1] in "+-"):
                j += 1
                if text[j] in "+-":
                    j += 1
                while j < n and text[j].isdigit():
                    j += 1
                kind = "DBL"
            num = text[i:j]
            if j < n and text[j] in "dD" and not (j + 1 < n and (text[j + 1].isalnum() or text[j + 1] == "_")):
                kind = "DBL"
                j += 1
            elif j < n and text[j] in "lL" and kind == "INT" and not (j + 1 < n and text[j + 1].isalnum()):
                j += 1
            toks.append((kind, num))
            i = j
            continue
        if ch.isalpha() or ch == "_":
            j = i
            while j < n and (text[j].isalnum() or text[j] == "_"):
                j += 1
            toks.append(("ID", text[i:j]))
            i = j
            continue
        for op in ("<=>", "<=", ">=", "!=", "<>", "==", "<", ">", "=", "(", ")", ",", "-", "+", "*", "/", "%"):
            if text.startswith(op, i):
                toks.append(("OP", op))
                i += len(op)
                break
        else:
            raise UnsupportedPredicate("unsupported character %r in %r" % (ch, text))
    toks.append(("EOF", ""))
    return toks


# ----------------------------------------------------------------------------- parser
class _Parser:
    def __init__(self, text: str):
        self.text = text
        self.toks = _tokenize(text)
        self.pos = 0

    def peek(self):
        return self.toks[self.pos]

    def take(self):
        t = self.toks[self.pos]
        self.pos += 1
        return t

    def keyword(self, word: str) -> bool:
        t = self.peek()
        if t[0] == "ID" and t[1].upper() == word:
            self.pos += 1
            return True
        return False

    def expect_op(self, op: str):
        t = self.take()
        if t != ("OP", op):
            raise PredicateSyntaxError("expected %r in %r" % (op, self.text))

    def parse(self):
        node = self.or_expr()
        if self.peek()[0] != "EOF":
            raise PredicateSyntaxError("unexpected %r in %r" % (self.peek()[1], self.text))
        return node

    def or_expr(self):
        node = self.and_expr()
        while self.keyword("OR"):
            node = ("or", node, self.and_expr())
        return node

    def and_expr(self):
        node = self.not_expr()
        while self.keyword("AND"):
            node = ("and", node, self.not_expr())
        return node

    def not_expr(self):
        if self.keyword("NOT"):
            return ("not", self.not_expr())
        return self.predicate()

    def predicate(self):
        left = self.value()
        t = self.peek()
        if t[0] == "OP" and t[1] in ("=", "==", "!=", "<>", "<", "<=", ">", ">=", "<=>"):
            self.take()
            op = {"==": "=", "<>": "!="}.get(t[1], t[1])
            return ("cmp", op, left, self.value())
        negated = self.keyword("NOT")
        if self.keyword("IN"):
            self.expect_op("(")
            items = [self.value()]
            while self.peek() == ("OP", ","):
                self.take()
                items.append(self.value())
            self.expect_op(")")
            node = ("in", left, items)
            return ("not", node) if negated else node
        if self.keyword("BETWEEN"):
            lo = self.value()
            if not self.keyword("AND"):
                raise PredicateSyntaxError("BETWEEN without AND in %r" % self.text)
            hi = self.value()
            node = ("and", ("cmp", ">=", left, lo), ("cmp", "<=", left, hi))
            return ("not", node) if negated else node
        if negated:
            raise PredicateSyntaxError("dangling NOT in %r" % self.text)
        if self.keyword("IS"):
            neg = self.keyword("NOT")
            if not self.keyword("NULL"):
                raise PredicateSyntaxError("expected NULL after IS in %r" % self.text)
            return ("isnotnull" if neg else "isnull", left)
        return ("truth", left)

    def value(self):
        node = self._operand()
        t = self.peek()
        if t[0] == "OP" and t[1] in ("+", "-", "*", "/", "%"):
            raise UnsupportedPredicate("arithmetic (%s) is not GPU-eligible in %r" % (t[1], self.text))
        return node

    def _operand(self):
        t = self.take()
        kind, text = t
        if kind == "OP" and text in ("-", "+"):
            inner = self._operand()
            if inner[0] != "lit" or inner[1] not in ("int", "dec", "dbl"):
                raise UnsupportedPredicate("unary %s on a non-literal in %r" % (text, self.text))
            if text == "-":
                return ("lit", inner[1], -inner[2])
            return inner
        if kind == "OP" and text == "(":
            node = self.or_expr()
            self.expect_op(")")
            return node
        if kind == "INT":
            return ("lit", "int", int(text))
        if kind == "DEC":
            return ("lit", "dec", Fraction(Decimal(text)))
        if kind == "DBL":
            return ("lit", "dbl", float(text))
        if kind == "STR":
            # Spark 2.2's grammar concatenates adjacent string literals (`constant: STRING+`), so
            # the 'a''b' that Check.isContainedIn writes for a quote (Check.scala:908-910) is "ab"
            while self.peek()[0] == "STR":
                text += self.take()[1]
            return ("lit", "str", text)
        if kind == "ID":
            up = text.upper()
            if up in ("TRUE", "FALSE"):
                return ("lit", "bool", up == "TRUE")
            if up == "NULL":
                return ("lit", "null", None)
            if self.peek() == ("OP", "(") and up == "CAST":
                self.take()
                inner = self.value()
                if not self.keyword("AS"):
                    raise PredicateSyntaxError("expected AS in CAST of %r" % self.text)
                t2 = self.take()
                if t2[0] != "ID":
                    raise PredicateSyntaxError("expected a type name in CAST of %r" % self.text)
                if self.peek() == ("OP", "("):  # DECIMAL(p, s), VARCHAR(n), ...
                    raise UnsupportedPredicate("CAST to %s(...) is not GPU-eligible" % t2[1])
                target = _CAST_TYPES.get(t2[1].upper())
                if target is None:
                    raise UnsupportedPredicate("CAST to %s is not GPU-eligible" % t2[1])
                self.expect_op(")")
                return ("cast", inner, target)
            if self.peek() == ("OP", "("):
                if up != "COALESCE":
                    raise UnsupportedPredicate("function %s() is not GPU-eligible" % text)
                self.take()
                args = [self.value()]
                while self.peek() == ("OP", ","):
                    self.take()
                    args.append(self.value())
                self.expect_op(")")
                return ("coalesce", args)
            return ("col", text)
        raise PredicateSyntaxError("unexpected token %r in %r" % (text, self.text))


# ----------------------------------------------------------------------------- typing/codegen
class _Compiler:
    def __init__(self, schema: Dict[str, Tuple[int, str]]):
        self.schema = schema  # name -> (batch column index, dtype)
        self.code: List[Insn] = []
        self.pool = bytearray()  # DQ_P_LIT_STRING bytes

    def column(self, name: str) -> Tuple[int, str]:
        return self.schema[resolve_column(name, self.schema)]

    def stype(self, node) -> str:
        """Spark type class of a value: int / f32 / f64 / dec / str / bool / null."""
        t = node[0]
        if t == "col":
            dtype = self.column(node[1])[1]
            return ("int" if dtype in _INTEGRAL else "f32" if dtype == "float32" else
                    "f64" if dtype == "float64" else "bool" if dtype == "bool" else "str")
        if t == "cast":
            return {"float32": "f32", "float64": "f64", "bool": "bool"}.get(node[2], "int")
        if t == "coalesce":
            kinds = {self.stype(a) for a in node[1]} - {"null"}
            if "str" in kinds:
                return "str"
            if "f64" in kinds or ("f32" in kinds and "dec" in kinds):
                return "f64"
            for k in ("f32", "dec", "int", "bool"):
                if k in kinds:
                    return k
            return "null"
        if t == "lit":
            return {"dbl": "f64"}.get(node[1], node[1])
        return "bool"

    def vtype(self, node) -> str:
        t = node[0]
        if t == "lit":
            return node[1]
        if t in ("col", "cast"):
            return {"f32": "dbl", "f64": "dbl"}.get(self.stype(node), self.stype(node))
        if t == "coalesce":
            kinds = [self.vtype(a) for a in node[1]]
            kinds = [k for k in kinds if k != "null"] or ["null"]
            for k in ("str", "dbl", "dec", "int", "bool"):
                if k in kinds:
                    if k == "dec" and "int" in kinds:
                        return "dec"
                    return k
            return "null"
        return "bool"

    def _has_f32(self, node) -> bool:
        """A FloatType value: a FLOAT column, a CAST to FLOAT, or a COALESCE typed FloatType."""
        return self.stype(node) == "f32"

    def emit(self, opcode, arg=0, i64=0, f64=0.0):
        self.code.append((opcode, arg, int(i64), float(f64)))

    def emit_value(self, node, target: str):
        """Push `node`; target is the comparison's type class (int / dbl / str, or f32: Spark
        coerces an integral operand to FloatType, so it is rounded to float first)."""
        t = node[0]
        if t == "col":
            idx, dtype = self.column(node[1])
            if dtype == "string" and target != "str":
                raise UnsupportedPredicate("string column %s in a numeric context" % node[1])
            self.emit(L.DQ_P_COLUMN, idx)
            if target == "f32" and dtype in _INTEGRAL | {"bool"}:
                self.emit(L.DQ_P_CAST, L.TYPE_CODES["float32"])
        elif t == "cast":
            inner, to = node[1], node[2]
            ik = self.stype(inner)
            if ik == "str":
                if to != "float64":
                    raise UnsupportedPredicate("CAST of a string to %s stays on Spark" % to)
                self.emit_value(inner, "str")
                self.emit(L.DQ_P_CAST_DOUBLE)
            elif ik == "dec":  # a decimal literal: Decimal.toDouble is correctly rounded
                if inner[0] != "lit" or to == "float32":
                    raise UnsupportedPredicate("CAST of a decimal-typed expression to %s" % to)
                v = inner[2]
                if to == "float64":
                    self.emit(L.DQ_P_LIT_FLOAT, f64=float(v))
                else:  # Decimal.toLong truncates toward zero (the low 64 bits); != 0 for boolean
                    w = (1 if v != 0 else 0) if to == "bool" else (math.trunc(v) + 2 ** 63) % 2 ** 64 - 2 ** 63
                    self.emit(L.DQ_P_LIT_INT, i64=w)
                    self.emit(L.DQ_P_CAST, L.TYPE_CODES[to])
            elif ik == "null":
                self.emit(L.DQ_P_LIT_NULL)
            else:
                self.emit_value(inner, "dbl" if ik in ("f32", "f64") else "int")
                self.emit(L.DQ_P_CAST, L.TYPE_CODES[to])
            if target == "f32" and to in _INTEGRAL | {"bool"}:
                self.emit(L.DQ_P_CAST, L.TYPE_CODES["float32"])
        elif t == "lit":
            kind, v = node[1], node[2]
            if kind == "null":
                self.emit(L.DQ_P_LIT_NULL)
            elif kind == "bool":
                self.emit(L.DQ_P_LIT_INT, i64=1 if v else 0)
                if target == "f32":
                    self.emit(L.DQ_P_CAST, L.TYPE_CODES["float32"])
            elif kind == "int":
                if target == "f32":
                    self.emit(L.DQ_P_LIT_FLOAT, f64=int_to_float32(v))
                elif target == "dbl":
                    self.emit(L.DQ_P_LIT_FLOAT, f64=float(v))
                else:
                    self.emit(L.DQ_P_LIT_INT, i64=v)
            elif kind == "dec":
                if target == "dbl":
                    self.emit(L.DQ_P_LIT_FLOAT, f64=float(v))
                elif v.denominator == 1 and -(2 ** 63) <= v.numerator < 2 ** 63:
                    self.emit(L.DQ_P_LIT_INT, i64=v.numerator)
                else:
                    raise UnsupportedPredicate("non-integral decimal in an integer context")
            elif kind == "dbl":
                self.emit(L.DQ_P_LIT_FLOAT, f64=v)
            elif target == "str":
                b = v.encode("utf-8")
                self.emit(L.DQ_P_LIT_STRING, len(b), i64=len(self.pool))
                self.pool += b
            else:
                raise UnsupportedPredicate("string literal in a numeric context")
        elif t == "coalesce":
            args = node[1]
            if target == "dbl" and self.stype(node) == "f32":  # COALESCE typed FloatType
                target = "f32"
            self.emit_value(args[0], target)
            for a in args[1:]:
                self.emit_value(a, target)
                self.emit(L.DQ_P_COALESCE)
        else:
            raise UnsupportedPredicate("boolean expression used as a value")

    _OPS = {"=": L.DQ_P_EQ, "!=": L.DQ_P_NE, "<": L.DQ_P_LT, "<=": L.DQ_P_LE, ">": L.DQ_P_GT,
            ">=": L.DQ_P_GE, "<=>": L.DQ_P_EQ_NULLSAFE}
    _FLIP = {"<": ">", "<=": ">=", ">": "<", ">=": "<=", "=": "=", "!=": "!=", "<=>": "<=>"}

    def emit_cmp(self, op, a, b):
        ta, tb = self.vtype(a), self.vtype(b)
        if ta == "str" and tb == "str":  # UTF8String.compareTo: byte-wise
            self.emit_value(a, "str")
            self.emit_value(b, "str")
            self.emit(self._OPS[op], L.DQ_CMP_AS_INT64)
            return
        if "str" in (ta, tb) and "null" not in (ta, tb):
            # Spark 2.2 PromoteStrings: a string compared with a number is Cast to DoubleType
            # (java.lang.Double.parseDouble of the trimmed text, NULL when unparsable) and the
            # comparison runs in double (e.g. `item > 3` on a string column, CheckTest.scala:193)
            if "bool" in (ta, tb):
                raise UnsupportedPredicate("comparison of a string with a boolean")
            for node, kind in ((a, ta), (b, tb)):
                if kind == "str":
                    self.emit_value(node, "str")
                    self.emit(L.DQ_P_CAST_DOUBLE)
                else:
                    self.emit_value(node, "dbl")
            self.emit(self._OPS[op], L.DQ_CMP_AS_FLOAT64)
            return
        if ta == "null" or tb == "null":
            if op == "<=>":  # x <=> NULL  ==  x IS NULL
                other = a if tb == "null" else b
                vt = self.vtype(other)
                self.emit_value(other, vt if vt in ("dbl", "str") else "int")
                self.emit(L.DQ_P_IS_NULL)
                return
            self.emit(L.DQ_P_LIT_NULL)  # any other comparison with NULL is NULL
            self.emit(L.DQ_P_LIT_NULL)
            self.emit(L.DQ_P_EQ, L.DQ_CMP_AS_INT64)
            return
        if "int" in (ta, tb) and (self._has_f32(a) or self._has_f32(b)):
            # Spark 2.2 coerces float vs int / long to FloatType: the integral side is rounded to
            # float first (a literal once on the host, anything else per row by DQ_P_CAST), then
            # compared in fp64, which orders float values as FloatType does
            self.emit_value(a, "f32")
            self.emit_value(b, "f32")
            self.emit(self._OPS[op], L.DQ_CMP_AS_FLOAT64)
            return
        if "dbl" in (ta, tb):
            self.emit_value(a, "dbl")
            self.emit_value(b, "dbl")
            self.emit(self._OPS[op], L.DQ_CMP_AS_FLOAT64)
            return
        if "dec" in (ta, tb):
            if ta == "dec" and tb == "dec" and a[0] == "lit" and b[0] == "lit":
                x, y = a[2], b[2]
                res = {"=": x == y, "!=": x != y, "<": x < y, "<=": x <= y, ">": x > y,
                       ">=": x >= y, "<=>": x == y}[op]
                self.emit(L.DQ_P_TRUE if res else L.DQ_P_FALSE)
                return
            if ta == "dec" and a[0] == "lit":  # literal on the left: flip
                a, b, ta, tb, op = b, a, tb, ta, self._FLIP[op]
            if b[0] != "lit":
                raise UnsupportedPredicate("decimal-typed expression")
            d = b[2]
            if d.denominator == 1:
                self.emit_value(a, "int")
                self.emit_value(b, "int")
                self.emit(self._OPS[op], L.DQ_CMP_AS_INT64)
                return
            # exact long-vs-decimal comparison for a non-integral decimal d
            lo, hi = math.floor(d), math.ceil(d)
            if op in ("<", "<="):
                self.emit_value(a, "int")
                self.emit(L.DQ_P_LIT_INT, i64=lo)
                self.emit(L.DQ_P_LE, L.DQ_CMP_AS_INT64)
            elif op in (">", ">="):
                self.emit_value(a, "int")
                self.emit(L.DQ_P_LIT_INT, i64=hi)
                self.emit(L.DQ_P_GE, L.DQ_CMP_AS_INT64)
            elif op in ("=", "!="):  # never equal: FALSE / TRUE, NULL when a is NULL
                self.emit_value(a, "int")
                self.emit_value(a, "int")
                self.emit(L.DQ_P_NE if op == "=" else L.DQ_P_EQ, L.DQ_CMP_AS_INT64)
            else:  # <=> never matches and is never NULL
                self.emit(L.DQ_P_FALSE)
            return
        self.emit_value(a, "int")
        self.emit_value(b, "int")
        self.emit(self._OPS[op], L.DQ_CMP_AS_INT64)

    def emit_bool(self, node):
        t = node[0]
        if t == "cmp":
            self.emit_cmp(node[1], node[2], node[3])
        elif t in ("and", "or"):
            self.emit_bool(node[1])
            self.emit_bool(node[2])
            self.emit(L.DQ_P_AND if t == "and" else L.DQ_P_OR)
        elif t == "not":
            self.emit_bool(node[1])
            self.emit(L.DQ_P_NOT)
        elif t in ("isnull", "isnotnull"):
            vt = self.vtype(node[1])
            if node[1][0] in ("col", "lit", "coalesce", "cast"):
                self.emit_value(node[1], vt if vt in ("dbl", "str") else "int")
            else:
                self.emit_bool(node[1])
            self.emit(L.DQ_P_IS_NULL if t == "isnull" else L.DQ_P_IS_NOT_NULL)
        elif t == "in":
            x, items = node[1], node[2]
            kinds = {self.vtype(v) for v in [x] + list(items)} - {"null"}
            if "str" in kinds and len(kinds) > 1:
                # Spark 2.2 InConversion widens a string/number IN list to StringType (string
                # comparison of the numbers' text), not to double as a plain comparison does
                raise UnsupportedPredicate("IN list mixing strings and numbers")
            for k, item in enumerate(items):
                self.emit_cmp("=", x, item)
                if k:
                    self.emit(L.DQ_P_OR)
        elif t == "truth":
            v = node[1]
            if v[0] == "lit" and v[1] == "bool":
                self.emit(L.DQ_P_TRUE if v[2] else L.DQ_P_FALSE)
            elif v[0] == "col" and self.vtype(v) == "bool":
                self.emit(L.DQ_P_COLUMN, self.column(v[1])[0])
            elif v[0] == "cast" and v[2] == "bool":
                self.emit_value(v, "int")
            elif v[0] in ("or", "and", "not", "cmp", "in", "isnull", "isnotnull", "truth"):
                self.emit_bool(v)
            else:
                raise UnsupportedPredicate("non-boolean predicate")
        else:
            raise UnsupportedPredicate("unsupported expression %s" % t)


def parse(text: str):
    return _Parser(text).parse()


def int_to_float32(v: int) -> float:
    """Java l2f / i2f: the integer rounded to the nearest float (ties to even), exactly."""
    if v == 0:
        return 0.0
    a = abs(v)
    sh = a.bit_length() - 24
    if sh > 0:
        q, rem = divmod(a, 1 << sh)
        half = 1 << (sh - 1)
        if rem > half or (rem == half and q & 1):
            q += 1
        a = q << sh
    return float(a if v > 0 else -a)


def resolve_column(name: str, schema) -> str:
    """Spark 2.2 resolves column references case-insensitively by default: the schema's own
    name for `name`.  KeyError when none matches (AnalysisException), ValueError when two
    columns match (an ambiguous reference)."""
    if name in schema and sum(1 for k in schema if k.lower() == name.lower()) == 1:
        return name
    hits = [k for k in schema if k.lower() == name.lower()]
    if not hits:
        raise KeyError(name)
    if len(hits) > 1:
        raise ValueError("Reference '%s' is ambiguous, could be: %s" % (name, ", ".join(sorted(hits))))
    return hits[0]


def referenced_columns(text: str) -> List[str]:
    out: List[str] = []

    def walk(node):
        if isinstance(node, tuple):
            if node and node[0] == "col":
                if node[1] not in out:
                    out.append(node[1])
                return
            for x in node[1:]:
                walk(x)
        elif isinstance(node, list):
            for x in node:
                walk(x)

    walk(parse(text))
    return out


class CompiledPredicate:
    """Postfix program + string pool, ready for a dq_predicate."""

    def __init__(self, code: List[Insn], pool: bytes):
        self.code = code
        self.pool = bytes(pool)

    def __iter__(self):  # (opcode, arg, i64, f64) tuples
        return iter(self.code)

    def __len__(self):
        return len(self.code)

    def __repr__(self):
        return "CompiledPredicate(%r, pool=%r)" % (self.code, self.pool)


def compile_predicate(text: str, schema: Dict[str, Tuple[int, str]]) -> CompiledPredicate:
    """Compile `text` against {column: (batch index, dtype)}.  Raises KeyError for unknown
    columns (Spark: AnalysisException), UnsupportedPredicate outside the GPU subset."""
    c = _Compiler(schema)
    c.emit_bool(parse(text))
    return CompiledPredicate(c.code, c.pool)
