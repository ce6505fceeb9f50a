"""Query model for the hot path (mirror of pinot-core's QueryContext / FilterContext / predicates) and a
parser for the SQL subset the reference's query tests use on this path:

  SELECT agg(col) [AS alias], ... FROM t [WHERE filter] [GROUP BY c1, ...] [ORDER BY x [ASC|DESC], ...]
  [LIMIT n] [OPTION(k=v, ...)]

filter: AND / OR / NOT / ( ) over  col = v | col != v | col <> v | col < v | col <= v | col > v | col >= v |
        col BETWEEN a AND b | col IN (...) | col NOT IN (...) | REGEXP_LIKE(col, 'regex') | col [NOT] LIKE 'pattern'
REGEXP_LIKE / LIKE become RegexpLikePredicate as in RequestContextUtils.java:231-236 (LIKE through likeToRegexpLike).
Comparison predicates become RangePredicate exactly as the reference's RequestContextUtils does
(pinot-common/.../request/context/RequestContextUtils.java: >, >=, <, <=, BETWEEN -> RANGE).
Aggregations: COUNT(*), SUM, MIN, MAX, AVG, MINMAXRANGE, DISTINCTCOUNT, DISTINCTSUM, DISTINCTAVG, DISTINCTCOUNTHLL(col[, log2m]), DISTINCTCOUNTRAWHLL(col[, log2m]) and their *MV
forms.
"""
import re
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

DEFAULT_HLL_LOG2M = 8          # CommonConstants.Helix.DEFAULT_HYPERLOGLOG_LOG2M
DEFAULT_NUM_GROUPS_LIMIT = 100_000   # InstancePlanMakerImplV2.DEFAULT_NUM_GROUPS_LIMIT
DEFAULT_MIN_SERVER_GROUP_TRIM_SIZE = 5000   # GroupByUtils.DEFAULT_MIN_NUM_GROUPS
UNBOUNDED = "*"                # RangePredicate.UNBOUNDED


# ------------------------------------------------------------------ predicates (pinot-common request/context)
@dataclass(frozen=True)
class EqPredicate:
    column: str
    value: object


@dataclass(frozen=True)
class NotEqPredicate:
    column: str
    value: object


@dataclass(frozen=True)
class InPredicate:
    column: str
    values: Tuple


@dataclass(frozen=True)
class NotInPredicate:
    column: str
    values: Tuple


@dataclass(frozen=True)
class RangePredicate:
    column: str
    lower: object = UNBOUNDED
    lower_inclusive: bool = False
    upper: object = UNBOUNDED
    upper_inclusive: bool = False


@dataclass(frozen=True)
class RegexpLikePredicate:
    """REGEXP_LIKE(col, pattern): a value matches when the pattern is found in it (Matcher.find(),
    RegexpLikePredicateEvaluatorFactory.java); LIKE arrives converted by like_to_regexp."""
    column: str
    pattern: str


def like_to_regexp(like):
    """RegexpPatternConverterUtils.likeToRegexpLike, restated from its test vectors (RegexpPatternConverterUtilsTest.java):
    leading / trailing '%' runs drop the '^' / '$' anchor, '%' -> '.*', '_' -> '.', a backslash escapes the next
    character (a trailing lone backslash is a literal one), regex metacharacters are escaped."""
    n = len(like)
    start, end = 0, n
    while start < end and like[start] == "%":
        start += 1
    while end > start and like[end - 1] == "%" and not (end - 2 >= start and like[end - 2] == "\\"):
        end -= 1
    out = ["^"] if start == 0 else []
    i = start
    while i < end:
        c = like[i]
        if c == "\\":
            if i + 1 < end:
                out.append("\\" + like[i + 1])
                i += 2
                continue
            out.append("\\\\")
        elif c == "%":
            out.append(".*")
        elif c == "_":
            out.append(".")
        elif c in ".^$*+?()[]{}|":
            out.append("\\" + c)
        else:
            out.append(c)
        i += 1
    if end == n:
        out.append("$")
    return "".join(out)


@dataclass(frozen=True)
class And:
    children: Tuple


@dataclass(frozen=True)
class Or:
    children: Tuple


@dataclass(frozen=True)
class Not:
    child: object


@dataclass(frozen=True)
class BoolFilter:
    """A constant filter (the boolean literal expression the reference's filter optimizers produce: TRUE becomes
    MatchAllFilterOperator, FALSE EmptyFilterOperator)."""
    value: bool


@dataclass(frozen=True)
class Comparison:
    """`a = b` / `a != b` where a side is not a plain column-vs-literal predicate (literal = literal, column = column):
    folded by IdenticalPredicateFilterOptimizer / constant evaluation (optimizer.py); each side ("id"|"lit", text)."""
    lhs: Tuple
    op: str
    rhs: Tuple


PREDICATES = (EqPredicate, NotEqPredicate, InPredicate, NotInPredicate, RangePredicate, RegexpLikePredicate)


# AggregationFunctionType names the hot path runs: single-value functions and their multi-value (*MV) forms, which
# aggregate every value of a multi-value column (SumMVAggregationFunction, CountMVAggregationFunction, ...)
SUPPORTED_FUNCTIONS = ("SUM", "MIN", "MAX", "AVG", "DISTINCTCOUNTHLL", "DISTINCTCOUNTRAWHLL", "MINMAXRANGE", "DISTINCTCOUNT",
                       "DISTINCTCOUNTBITMAP", "DISTINCTCOUNTBITMAPMV",
                       "DISTINCTSUM", "DISTINCTAVG",
                       "COUNTMV", "SUMMV", "MINMV", "MAXMV", "AVGMV", "DISTINCTCOUNTHLLMV", "DISTINCTCOUNTRAWHLLMV",
                       "MINMAXRANGEMV",
                       "DISTINCTCOUNTMV", "DISTINCTSUMMV", "DISTINCTAVGMV")
# BaseDistinctAggregateAggregationFunction subclasses: the intermediate result is the set of distinct values (one
# presence accumulator on the GPU); they differ only in extractFinalResult (size / sum / average)
DISTINCT_SET_FUNCTIONS = ("DISTINCTCOUNT", "DISTINCTSUM", "DISTINCTAVG", "DISTINCTCOUNTBITMAP", "DISTINCTCOUNTMV",
                          "DISTINCTCOUNTBITMAPMV", "DISTINCTSUMMV",
                          "DISTINCTAVGMV")


# DistinctCountBitmapAggregationFunction: the same value presence per group, reported as the set of the values' Java
# hash codes (its RoaringBitmap: java_hash.py), so equal hash codes count once
BITMAP_FUNCTIONS = ("DISTINCTCOUNTBITMAP", "DISTINCTCOUNTBITMAPMV")

# HyperLogLog functions: one register set per group (DistinctCountHLLAggregationFunction); the RAW forms differ only in
# the final result, the serialized registers (DistinctCountRawHLLAggregationFunction: SerializedHLL.toString, the hex
# of HyperLogLog.getBytes)
HLL_FUNCTIONS = ("DISTINCTCOUNTHLL", "DISTINCTCOUNTHLLMV", "DISTINCTCOUNTRAWHLL", "DISTINCTCOUNTRAWHLLMV")


def base_function(fn):
    """Merge/extract semantics of a function: the *MV forms behave like their single-value form, COUNTMV like COUNT."""
    return fn[:-2] if fn.endswith("MV") else fn


@dataclass(frozen=True)
class Aggregation:
    function: str              # COUNT SUM MIN MAX AVG DISTINCTCOUNTHLL and the *MV forms
    column: Optional[str] = None
    log2m: int = DEFAULT_HLL_LOG2M

    @property
    def result_name(self):
        """AggregationFunction.getResultColumnName: lower-case function name + (column)."""
        if self.function == "COUNT":
            return "count(*)"
        return "%s(%s)" % (self.function.lower(), self.column)


@dataclass(frozen=True)
class OrderBy:
    expr: object               # Aggregation or column name
    asc: bool = True


@dataclass
class Query:
    aggregations: List[Aggregation]
    aliases: List[Optional[str]] = field(default_factory=list)
    filter: object = None
    group_by: List[str] = field(default_factory=list)
    order_by: List[OrderBy] = field(default_factory=list)
    limit: int = 10
    options: dict = field(default_factory=dict)
    select_columns: List[str] = field(default_factory=list)
    num_select_aggs: int = -1   # aggregations after this index are ORDER BY-only

    @property
    def num_groups_limit(self):
        return int(self.options.get("numGroupsLimit", DEFAULT_NUM_GROUPS_LIMIT))

    @property
    def min_server_group_trim_size(self):
        return int(self.options.get("minServerGroupTrimSize", DEFAULT_MIN_SERVER_GROUP_TRIM_SIZE))

    def columns(self):
        cols = set(self.group_by)
        for a in self.aggregations:
            if a.column:
                cols.add(a.column)

        def walk(f):
            if f is None:
                return
            if isinstance(f, (And, Or)):
                for c in f.children:
                    walk(c)
            elif isinstance(f, Not):
                walk(f.child)
            elif hasattr(f, "column"):
                cols.add(f.column)
        walk(self.filter)
        return cols


# ------------------------------------------------------------------ SQL subset parser
_TOKEN = re.compile(r"\s*(?:(?P<num>-?\d+(?:\.\d+)?(?:[eE][-+]?\d+)?)|(?P<str>'(?:[^']|'')*')|"
                    r"(?P<qid>\"(?:[^\"]|\"\")*\")|"
                    r"(?P<op><>|!=|<=|>=|=|<|>|\(|\)|,|\*)|(?P<id>[A-Za-z_][A-Za-z0-9_\.]*))")


def _tokenize(sql):
    pos, out = 0, []
    sql = sql.strip().rstrip(";")
    while pos < len(sql):
        m = _TOKEN.match(sql, pos)
        if not m or m.end() == pos:
            raise ValueError("cannot tokenize at: %r" % sql[pos:pos + 20])
        pos = m.end()
        if m.group("num") is not None:
            out.append(("lit", m.group("num")))
        elif m.group("str") is not None:
            out.append(("lit", m.group("str")[1:-1].replace("''", "'")))
        elif m.group("qid") is not None:  # "quoted identifier"
            out.append(("id", m.group("qid")[1:-1].replace('""', '"')))
        elif m.group("op") is not None:
            out.append(("op", m.group("op")))
        else:
            out.append(("id", m.group("id")))
    return out


class _Parser:
    def __init__(self, sql):
        self.t = _tokenize(sql)
        self.i = 0

    def peek(self, k=0):
        return self.t[self.i + k] if self.i + k < len(self.t) else (None, None)

    def kw(self, word):
        tok = self.peek()
        if tok[0] == "id" and tok[1].upper() == word:
            self.i += 1
            return True
        return False

    def expect_kw(self, word):
        if not self.kw(word):
            raise ValueError("expected %s at token %r" % (word, self.peek()))

    def op(self, sym):
        tok = self.peek()
        if tok[0] == "op" and tok[1] == sym:
            self.i += 1
            return True
        return False

    def expect_op(self, sym):
        if not self.op(sym):
            raise ValueError("expected %r at token %r" % (sym, self.peek()))

    def ident(self):
        tok = self.peek()
        if tok[0] != "id":
            raise ValueError("expected identifier at %r" % (tok,))
        self.i += 1
        return tok[1]

    def literal(self):
        tok = self.peek()
        if tok[0] != "lit":
            raise ValueError("expected literal at %r" % (tok,))
        self.i += 1
        return tok[1]

    # SELECT list item
    def aggregation(self):
        fn = self.ident().upper()
        self.expect_op("(")
        if self.kw("DISTINCT"):
            # CalciteSqlParser.java:761-772: COUNT / SUM / AVG (DISTINCT x) -> DISTINCTCOUNT / DISTINCTSUM / DISTINCTAVG,
            # any other aggregation on DISTINCT is refused
            if fn not in ("COUNT", "SUM", "AVG"):
                raise ValueError("Function '%s' on DISTINCT is not supported." % fn)
            fn = "DISTINCT" + fn
        elif fn == "COUNT":
            self.expect_op("*")
            self.expect_op(")")
            return Aggregation("COUNT")
        col = self.ident()
        log2m = DEFAULT_HLL_LOG2M
        if self.op(","):
            log2m = int(self.literal())
        self.expect_op(")")
        if fn not in SUPPORTED_FUNCTIONS:
            raise ValueError("unsupported aggregation %s" % fn)
        return Aggregation(fn, col, log2m)

    def filter_or(self):
        left = self.filter_and()
        items = [left]
        while self.kw("OR"):
            items.append(self.filter_and())
        return items[0] if len(items) == 1 else Or(tuple(items))

    def filter_and(self):
        items = [self.filter_not()]
        while self.kw("AND"):
            items.append(self.filter_not())
        return items[0] if len(items) == 1 else And(tuple(items))

    def filter_not(self):
        if self.kw("NOT"):
            return Not(self.filter_not())
        if self.op("("):
            f = self.filter_or()
            self.expect_op(")")
            return f
        return self.predicate()

    def predicate(self):
        tok, nxt = self.peek(), self.peek(1)
        if tok[0] == "id" and tok[1].upper() in ("TRUE", "FALSE") and not (nxt[0] == "op" and nxt[1] in
                                                                           ("=", "!=", "<>", "<", "<=", ">", ">=")):
            self.i += 1
            return BoolFilter(tok[1].upper() == "TRUE")
        if tok[0] == "lit" or (tok[0] == "id" and nxt[0] == "op" and nxt[1] in ("=", "!=", "<>") and
                               self.peek(2)[0] == "id" and self.peek(2)[1].upper() not in ("TRUE", "FALSE")):
            # literal = literal, column = column: a comparison the filter optimizers fold (optimizer.py)
            lhs = (tok[0], tok[1])
            self.i += 1
            op = self.peek()
            if op[0] != "op" or op[1] not in ("=", "!=", "<>"):
                raise ValueError("expected = or != after %r" % (tok,))
            self.i += 1
            rhs = self.peek()
            if rhs[0] not in ("id", "lit"):
                raise ValueError("expected a literal or column at %r" % (rhs,))
            self.i += 1
            return Comparison(lhs, "=" if op[1] == "=" else "!=", (rhs[0], rhs[1]))
        if tok[0] == "id" and tok[1].upper() == "REGEXP_LIKE" and nxt == ("op", "("):
            self.i += 2
            col = self.ident()
            self.expect_op(",")
            pat = self.literal()
            self.expect_op(")")
            return RegexpLikePredicate(col, str(pat))
        col = self.ident()
        if self.kw("BETWEEN"):
            lo = self.literal()
            self.expect_kw("AND")
            hi = self.literal()
            return RangePredicate(col, lo, True, hi, True)
        negate = self.kw("NOT")
        if self.kw("LIKE"):
            f = RegexpLikePredicate(col, like_to_regexp(str(self.literal())))
            return Not(f) if negate else f
        if self.kw("IN"):
            self.expect_op("(")
            vals = [self.literal()]
            while self.op(","):
                vals.append(self.literal())
            self.expect_op(")")
            return NotInPredicate(col, tuple(vals)) if negate else InPredicate(col, tuple(vals))
        if negate:
            raise ValueError("NOT must be followed by IN or LIKE here")
        tok = self.peek()
        if tok[0] != "op":
            raise ValueError("expected comparison at %r" % (tok,))
        self.i += 1
        v = self.literal()
        return {
            "=": lambda: EqPredicate(col, v),
            "!=": lambda: NotEqPredicate(col, v),
            "<>": lambda: NotEqPredicate(col, v),
            "<": lambda: RangePredicate(col, UNBOUNDED, False, v, False),
            "<=": lambda: RangePredicate(col, UNBOUNDED, False, v, True),
            ">": lambda: RangePredicate(col, v, False, UNBOUNDED, False),
            ">=": lambda: RangePredicate(col, v, True, UNBOUNDED, False),
        }[tok[1]]()

    def parse(self):
        self.expect_kw("SELECT")
        aggs, aliases, plain_cols = [], [], []
        while True:
            tok, nxt = self.peek(), self.peek(1)
            if tok[0] == "id" and not (nxt[0] == "op" and nxt[1] == "("):
                plain_cols.append(self.ident())  # group-by column in the select list
            else:
                aggs.append(self.aggregation())
                aliases.append(self.ident() if self.kw("AS") else None)
            if not self.op(","):
                break
        self.expect_kw("FROM")
        self.ident()
        q = Query(aggregations=aggs, aliases=aliases)
        q.select_columns = plain_cols
        q.num_select_aggs = len(aggs)
        if self.kw("WHERE"):
            q.filter = self.filter_or()
        if self.kw("GROUP"):
            self.expect_kw("BY")
            q.group_by.append(self.ident())
            while self.op(","):
                q.group_by.append(self.ident())
        if self.kw("ORDER"):
            self.expect_kw("BY")
            while True:
                tok, nxt = self.peek(), self.peek(1)
                if tok[0] == "id" and nxt[0] == "op" and nxt[1] == "(":
                    expr = self.aggregation()
                    if expr not in aggs:  # ORDER BY aggregation absent from the select list: computed, not output
                        aggs.append(expr)
                        aliases.append(None)
                else:
                    name = self.ident()
                    expr = name
                    for a, al in zip(aggs, aliases):
                        if al == name:
                            expr = a
                asc = True
                if self.kw("DESC"):
                    asc = False
                else:
                    self.kw("ASC")
                q.order_by.append(OrderBy(expr, asc))
                if not self.op(","):
                    break
        if self.kw("LIMIT"):
            q.limit = int(self.literal())
        if self.kw("TOP"):
            q.limit = int(self.literal())
        if self.kw("OPTION"):
            self.expect_op("(")
            while True:
                k = self.ident()
                self.expect_op("=")
                tok = self.peek()
                self.i += 1
                q.options[k] = tok[1]
                if not self.op(","):
                    break
            self.expect_op(")")
        if self.peek()[0] is not None:
            raise ValueError("trailing tokens: %r" % (self.t[self.i:],))
        return q


def parse_sql(sql: str) -> Query:
    return _Parser(sql).parse()


def parse_filter(text: str):
    """A WHERE clause on its own (the filter tree parse_sql builds for it)."""
    p = _Parser(text)
    f = p.filter_or()
    if p.peek()[0] is not None:
        raise ValueError("trailing tokens: %r" % (p.t[p.i:],))
    return f


def query_columns(query):
    """Every column a query reads: filter leaves, group-by columns, aggregation columns."""
    names = []

    def walk(f):
        for c in getattr(f, "children", ()) or ():
            walk(c)
        if getattr(f, "child", None) is not None:
            walk(f.child)
        if getattr(f, "column", None) is not None and f.column not in names:
            names.append(f.column)
    if query.filter is not None:
        walk(query.filter)
    for n in list(query.group_by) + [a.column for a in query.aggregations if a.column]:
        if n not in names:
            names.append(n)
    return names
