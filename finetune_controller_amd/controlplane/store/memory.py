"""In-memory MongoDB subset: collections with Motor-style async methods and an aggregation engine.

It implements exactly what the job store uses -- including the aggregation-derived fields the UI
depends on (``start_time`` / ``end_time`` / ``duration`` / ``status_merged`` computed by ``$addFields``
with ``$cond`` / ``$ifNull`` / ``$subtract``, the ``$setWindowFields`` ``$documentNumber`` row index and the
``$lookup`` + ``$map`` of dataset job names; ``/root/reference/app/database/db.py:282-679``) -- so the
same ``JobStore`` code runs against MongoDB (pymongo ``AsyncMongoClient``) or this engine.

Supported: filters with equality, dotted paths, ``$regex``/``$options``, ``$in``, ``$nin``, ``$ne``,
``$exists``, ``$lt/$lte/$gt/$gte``, ``$or``/``$and``; updates ``$set``, ``$unset``, ``$addToSet``,
``$push``, ``$inc`` (+ upsert); stages ``$match``, ``$addFields``/``$set``, ``$setWindowFields``
(``$documentNumber``), ``$sort``, ``$skip``, ``$limit``, ``$lookup``, ``$unset``, ``$project`` (inclusion),
``$count``; expressions ``$cond``, ``$eq``, ``$ne``, ``$gt``, ``$lt``, ``$and``, ``$or``, ``$not``,
``$ifNull``, ``$subtract``, ``$add``, ``$map``, ``$literal``.
"""
from __future__ import annotations

import copy
import datetime as _dt
import re
import threading
from dataclasses import dataclass
from typing import Any

from bson import ObjectId

_MISSING = object()


class DuplicateKeyError(Exception):
    pass


def _get(doc, path: str):
    cur = doc
    for part in path.split("."):
        if isinstance(cur, dict) and part in cur:
            cur = cur[part]
        elif isinstance(cur, list) and part.isdigit() and int(part) < len(cur):
            cur = cur[int(part)]
        else:
            return _MISSING
    return cur


def _set(doc, path: str, value):
    parts = path.split(".")
    cur = doc
    for p in parts[:-1]:
        if not isinstance(cur.get(p), dict):
            cur[p] = {}
        cur = cur[p]
    cur[parts[-1]] = value


def _unset(doc, path: str):
    parts = path.split(".")
    cur = doc
    for p in parts[:-1]:
        cur = cur.get(p)
        if not isinstance(cur, dict):
            return
    cur.pop(parts[-1], None)


def _norm(v):
    """Comparable form (tz-naive datetimes are treated as UTC, like MongoDB)."""
    if isinstance(v, _dt.datetime) and v.tzinfo is None:
        return v.replace(tzinfo=_dt.timezone.utc)
    if hasattr(v, "value") and v.__class__.__module__ != "builtins" and isinstance(getattr(v, "value"), str):
        return v.value  # str Enum
    return v


def _eq(a, b) -> bool:
    return _norm(a) == _norm(b)


def _cmp_key(v):
    v = _norm(v)
    if v is None or v is _MISSING:
        return (0, 0)
    if isinstance(v, bool):
        return (3, int(v))
    if isinstance(v, (int, float)):
        return (1, v)
    if isinstance(v, str):
        return (2, v)
    if isinstance(v, _dt.datetime):
        return (4, v.timestamp())
    if isinstance(v, ObjectId):
        return (5, str(v))
    return (6, str(v))


# ------------------------------------------------------------------ filters
def match(doc: dict, flt: dict) -> bool:
    for k, cond in flt.items():
        if k == "$or":
            if not any(match(doc, c) for c in cond):
                return False
            continue
        if k == "$and":
            if not all(match(doc, c) for c in cond):
                return False
            continue
        val = _get(doc, k)
        if isinstance(cond, dict) and any(str(x).startswith("$") for x in cond):
            if not _match_ops(val, cond):
                return False
        else:
            if isinstance(val, list) and not isinstance(cond, list):
                if not any(_eq(v, cond) for v in val):
                    return False
            elif val is _MISSING:
                if cond is not None:
                    return False
            elif not _eq(val, cond):
                return False
    return True


def _match_ops(val, ops: dict) -> bool:
    for op, arg in ops.items():
        if op == "$regex":
            flags = re.I if "i" in ops.get("$options", "") else 0
            if val is _MISSING or not isinstance(val, str) or not re.search(arg, val, flags):
                return False
        elif op == "$options":
            continue
        elif op == "$in":
            vals = val if isinstance(val, list) else [val]
            if not any(_eq(v, a) for v in vals for a in arg):
                return False
        elif op == "$nin":
            vals = val if isinstance(val, list) else [val]
            if any(_eq(v, a) for v in vals for a in arg):
                return False
        elif op == "$ne":
            if val is not _MISSING and _eq(val, arg):
                return False
        elif op == "$eq":
            if not _eq(val, arg):
                return False
        elif op == "$exists":
            if (val is not _MISSING) != bool(arg):
                return False
        elif op in ("$lt", "$lte", "$gt", "$gte"):
            if val is _MISSING or val is None:
                return False
            a, b = _cmp_key(val), _cmp_key(arg)
            if a[0] != b[0]:
                return False
            ok = {"$lt": a < b, "$lte": a <= b, "$gt": a > b, "$gte": a >= b}[op]
            if not ok:
                return False
        else:
            raise NotImplementedError(f"query operator {op}")
    return True


# ------------------------------------------------------------------ expressions
def evaluate(expr, doc, vars_: dict | None = None):
    vars_ = vars_ or {}
    if isinstance(expr, str):
        if expr.startswith("$$"):
            name, _, rest = expr[2:].partition(".")
            base = vars_.get(name, _MISSING)
            if not rest:
                return base
            v = _get(base, rest) if isinstance(base, dict) else _MISSING
            return v
        if expr.startswith("$"):
            return _get(doc, expr[1:])
        return expr
    if isinstance(expr, list):
        return [evaluate(e, doc, vars_) for e in expr]
    if isinstance(expr, dict):
        if len(expr) == 1:
            (op, arg), = expr.items()
            if op.startswith("$"):
                return _eval_op(op, arg, doc, vars_)
        return {k: evaluate(v, doc, vars_) for k, v in expr.items()}
    return expr


def _truthy(v) -> bool:
    return not (v is _MISSING or v is None or v is False or v == 0)


def _val(v):
    return None if v is _MISSING else v


def _eval_op(op, arg, doc, vs):
    ev = lambda e: evaluate(e, doc, vs)  # noqa: E731
    if op == "$cond":
        if isinstance(arg, list):
            c, t, f = arg
        else:
            c, t, f = arg["if"], arg["then"], arg["else"]
        return ev(t) if _truthy(ev(c)) else ev(f)
    if op == "$eq":
        a, b = (ev(x) for x in arg)
        return _eq(_val(a), _val(b))
    if op == "$ne":
        a, b = (ev(x) for x in arg)
        return not _eq(_val(a), _val(b))
    if op in ("$gt", "$lt", "$gte", "$lte"):
        a, b = (_cmp_key(_val(ev(x))) for x in arg)
        return {"$gt": a > b, "$lt": a < b, "$gte": a >= b, "$lte": a <= b}[op]
    if op == "$and":
        return all(_truthy(ev(x)) for x in arg)
    if op == "$or":
        return any(_truthy(ev(x)) for x in arg)
    if op == "$not":
        return not _truthy(ev(arg[0] if isinstance(arg, list) else arg))
    if op == "$ifNull":
        *cands, default = arg
        for c in cands:
            v = ev(c)
            if v is not _MISSING and v is not None:
                return v
        return ev(default)
    if op == "$subtract":
        a, b = (_norm(_val(ev(x))) for x in arg)
        if a is None or b is None:
            return None
        if isinstance(a, _dt.datetime) and isinstance(b, _dt.datetime):
            return int((a - b).total_seconds() * 1000)  # MongoDB: milliseconds
        if isinstance(a, _dt.datetime):
            return a - _dt.timedelta(milliseconds=b)
        return a - b
    if op == "$add":
        vals = [_norm(_val(ev(x))) for x in arg]
        if any(v is None for v in vals):
            return None
        dts = [v for v in vals if isinstance(v, _dt.datetime)]
        if dts:
            ms = sum(v for v in vals if not isinstance(v, _dt.datetime))
            return dts[0] + _dt.timedelta(milliseconds=ms)
        return sum(vals)
    if op == "$map":
        inp = ev(arg["input"])
        name = arg.get("as", "this")
        if inp is _MISSING or inp is None:
            return None
        return [evaluate(arg["in"], doc, {**vs, name: item}) for item in inp]
    if op == "$literal":
        return arg
    raise NotImplementedError(f"expression operator {op}")


# ------------------------------------------------------------------ update
def apply_update(doc: dict, upd: dict) -> bool:
    before = copy.deepcopy(doc)
    for op, fields in upd.items():
        if op == "$set":
            for k, v in fields.items():
                _set(doc, k, copy.deepcopy(v))
        elif op == "$unset":
            for k in fields:
                _unset(doc, k)
        elif op == "$addToSet":
            for k, v in fields.items():
                cur = _get(doc, k)
                cur = [] if cur is _MISSING or cur is None else list(cur)
                items = v["$each"] if isinstance(v, dict) and "$each" in v else [v]
                for it in items:
                    if not any(_eq(it, c) for c in cur):
                        cur.append(it)
                _set(doc, k, cur)
        elif op == "$push":
            for k, v in fields.items():
                cur = _get(doc, k)
                cur = [] if cur is _MISSING or cur is None else list(cur)
                cur.extend(v["$each"] if isinstance(v, dict) and "$each" in v else [v])
                _set(doc, k, cur)
        elif op == "$inc":
            for k, v in fields.items():
                cur = _get(doc, k)
                _set(doc, k, (0 if cur is _MISSING else cur) + v)
        else:
            raise NotImplementedError(f"update operator {op}")
    return doc != before


# ------------------------------------------------------------------ results / cursors
@dataclass
class InsertOneResult:
    inserted_id: Any


@dataclass
class UpdateResult:
    matched_count: int
    modified_count: int
    upserted_id: Any = None


@dataclass
class DeleteResult:
    deleted_count: int


class MemoryCursor:
    def __init__(self, docs):
        self._docs = docs
        self._i = 0

    def __aiter__(self):
        return self

    async def __anext__(self):
        if self._i >= len(self._docs):
            raise StopAsyncIteration
        d = self._docs[self._i]
        self._i += 1
        return d

    async def to_list(self, length=None):
        rest = self._docs[self._i:]
        if length is not None:
            rest = rest[:length]
        self._i += len(rest)
        return rest

    def sort(self, key, direction=1):
        self._docs.sort(key=lambda d: _cmp_key(_get(d, key)), reverse=direction < 0)
        return self


class MemoryCollection:
    def __init__(self, db: "MemoryDatabase", name: str):
        self.db, self.name = db, name
        self.docs: list[dict] = []
        self.unique: list[str] = []

    # ---- writes ----
    async def insert_one(self, doc: dict):
        with self.db.lock:
            if "_id" not in doc:
                doc["_id"] = ObjectId()
            for f in self.unique + ["_id"]:
                v = _get(doc, f)
                if v is not _MISSING and any(_eq(_get(d, f), v) for d in self.docs):
                    raise DuplicateKeyError(f"E11000 duplicate key {self.name}.{f}: {v}")
            self.docs.append(copy.deepcopy(doc))
            return InsertOneResult(doc["_id"])

    async def update_one(self, flt: dict, upd: dict, upsert: bool = False):
        with self.db.lock:
            for d in self.docs:
                if match(d, flt):
                    changed = apply_update(d, upd)
                    return UpdateResult(1, int(changed))
            if upsert:
                new = {k: v for k, v in flt.items() if not k.startswith("$") and not isinstance(v, dict)}
                apply_update(new, upd)
                r = await self.insert_one(new)
                return UpdateResult(0, 0, r.inserted_id)
            return UpdateResult(0, 0)

    async def update_many(self, flt: dict, upd: dict):
        with self.db.lock:
            n = m = 0
            for d in self.docs:
                if match(d, flt):
                    n += 1
                    m += int(apply_update(d, upd))
            return UpdateResult(n, m)

    async def delete_one(self, flt: dict):
        with self.db.lock:
            for i, d in enumerate(self.docs):
                if match(d, flt):
                    del self.docs[i]
                    return DeleteResult(1)
            return DeleteResult(0)

    async def delete_many(self, flt: dict):
        with self.db.lock:
            keep = [d for d in self.docs if not match(d, flt)]
            n = len(self.docs) - len(keep)
            self.docs = keep
            return DeleteResult(n)

    async def create_index(self, keys, unique: bool = False, **kw):
        if unique and isinstance(keys, str):
            self.unique.append(keys)
        return keys if isinstance(keys, str) else "_".join(f"{k}_{v}" for k, v in keys)

    # ---- reads ----
    async def find_one(self, flt: dict | None = None):
        with self.db.lock:
            for d in self.docs:
                if match(d, flt or {}):
                    return copy.deepcopy(d)
            return None

    def find(self, flt: dict | None = None):
        with self.db.lock:
            return MemoryCursor([copy.deepcopy(d) for d in self.docs if match(d, flt or {})])

    async def count_documents(self, flt: dict):
        with self.db.lock:
            return sum(1 for d in self.docs if match(d, flt))

    def aggregate(self, pipeline: list[dict]):
        with self.db.lock:
            docs = [copy.deepcopy(d) for d in self.docs]
            for stage in pipeline:
                docs = self.db._stage(docs, stage)
            return MemoryCursor(docs)


class MemoryDatabase:
    def __init__(self):
        self.lock = threading.RLock()
        self.collections: dict[str, MemoryCollection] = {}

    def __getitem__(self, name):
        if name not in self.collections:
            self.collections[name] = MemoryCollection(self, name)
        return self.collections[name]

    __getattr__ = lambda self, name: self[name] if not name.startswith("_") else object.__getattribute__(self, name)  # noqa: E731

    def _stage(self, docs, stage):
        (op, arg), = stage.items()
        if op == "$match":
            return [d for d in docs if match(d, arg)]
        if op in ("$addFields", "$set"):
            out = []
            for d in docs:
                vals = {k: evaluate(v, d) for k, v in arg.items()}
                for k, v in vals.items():
                    if v is _MISSING:
                        _unset(d, k)
                    else:
                        _set(d, k, v)
                out.append(d)
            return out
        if op == "$setWindowFields":
            order = _sorted(docs, arg.get("sortBy", {}))
            for i, d in enumerate(order):
                for field, spec in arg["output"].items():
                    if "$documentNumber" in spec:
                        d[field] = i + 1
                    else:
                        raise NotImplementedError(f"window {spec}")
            return docs
        if op == "$sort":
            return _sorted(docs, arg)
        if op == "$skip":
            return docs[arg:]
        if op == "$limit":
            return docs[:arg]
        if op == "$unset":
            for d in docs:
                for f in ([arg] if isinstance(arg, str) else arg):
                    _unset(d, f)
            return docs
        if op == "$project":
            out = []
            for d in docs:
                keep_id = arg.get("_id", 1)
                nd = {}
                for k, v in arg.items():
                    if k == "_id":
                        continue
                    if v in (1, True):
                        x = _get(d, k)
                        if x is not _MISSING:
                            _set(nd, k, x)
                    else:
                        _set(nd, k, evaluate(v, d))
                if keep_id and "_id" in d:
                    nd["_id"] = d["_id"]
                out.append(nd)
            return out
        if op == "$lookup":
            other = self[arg["from"]].docs
            out = []
            for d in docs:
                lv = _get(d, arg["localField"])
                lvs = lv if isinstance(lv, list) else [lv]
                d[arg["as"]] = [copy.deepcopy(o) for o in other
                                if any(_eq(_get(o, arg["foreignField"]), x) for x in lvs)]
                out.append(d)
            return out
        if op == "$count":
            return [{arg: len(docs)}]
        if op == "$group":
            return _group(docs, arg)
        raise NotImplementedError(f"aggregation stage {op}")


def _group(docs, spec: dict):
    """``$group`` with accumulators $sum / $avg / $min / $max / $first / $last / $push (what
    pymongo's ``count_documents`` sends is ``{"_id": 1, "n": {"$sum": 1}}``)."""
    groups: dict = {}
    order = []
    for d in docs:
        key = evaluate(spec["_id"], d) if spec["_id"] is not None else None
        hk = repr(key)
        if hk not in groups:
            groups[hk] = {"_id": key, "_acc": {f: [] for f in spec if f != "_id"}}
            order.append(hk)
        for f, acc in spec.items():
            if f == "_id":
                continue
            (aop, expr), = acc.items()
            v = evaluate(expr, d)
            groups[hk]["_acc"][f].append(None if v is _MISSING else v)
    out = []
    for hk in order:
        g = groups[hk]
        row = {"_id": g["_id"]}
        for f, acc in spec.items():
            if f == "_id":
                continue
            (aop, _), = acc.items()
            vals = g["_acc"][f]
            nums = [v for v in vals if isinstance(v, (int, float)) and not isinstance(v, bool)]
            present = [v for v in vals if v is not None]
            if aop == "$sum":
                row[f] = sum(nums)
            elif aop == "$avg":
                row[f] = sum(nums) / len(nums) if nums else None
            elif aop == "$min":
                row[f] = min(present, key=_cmp_key) if present else None
            elif aop == "$max":
                row[f] = max(present, key=_cmp_key) if present else None
            elif aop == "$first":
                row[f] = vals[0] if vals else None
            elif aop == "$last":
                row[f] = vals[-1] if vals else None
            elif aop == "$push":
                row[f] = present
            else:
                raise NotImplementedError(f"$group accumulator {aop}")
        out.append(row)
    return out


def _sorted(docs, spec: dict):
    out = list(docs)
    for key, direction in reversed(list(spec.items())):
        out.sort(key=lambda d: _cmp_key(_get(d, key)), reverse=direction < 0)
    return out


class MemoryClient:
    """``AsyncMongoClient`` look-alike."""

    def __init__(self):
        self.dbs: dict[str, MemoryDatabase] = {}

    def __getitem__(self, name):
        if name not in self.dbs:
            self.dbs[name] = MemoryDatabase()
        return self.dbs[name]

    async def close(self):
        return None
