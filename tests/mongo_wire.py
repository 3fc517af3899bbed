"""A MongoDB wire-protocol endpoint backed by the in-memory engine (store/memory.py), for driving the
real ``pymongo`` client -- BSON encoding, OP_MSG / OP_QUERY framing, handshake, command shapes,
cursors, write errors -- through the JobStore's production path without a mongod.

Supported: the handshake (``hello`` / ``isMaster`` over OP_QUERY or OP_MSG), ``ping``, ``buildInfo``,
``endSessions``, ``createIndexes``, ``insert``, ``update`` (``$set`` / ``$addToSet`` / ... as the engine
implements them, ``upsert``, ``multi``), ``delete``, ``find`` (filter, sort, skip, limit, projection
of included fields), ``aggregate`` (the engine's pipeline stages, ``count_documents``'
``$group``/``$sum`` form) and ``getMore``/``killCursors`` for single-batch cursors.  Duplicate keys come
back as write errors with code 11000, as from a real server.
"""
from __future__ import annotations

import asyncio
import datetime as dt
import socket
import struct
import threading

import bson
from bson.codec_options import CodecOptions

from finetune_controller_amd.controlplane.store.memory import DuplicateKeyError, MemoryClient

OP_REPLY, OP_QUERY, OP_MSG = 1, 2004, 2013
_CODEC = CodecOptions(tz_aware=True, tzinfo=dt.timezone.utc)


class MongoWireServer:
    def __init__(self):
        self.client = MemoryClient()
        self.loop = asyncio.new_event_loop()
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.sock.bind(("127.0.0.1", 0))
        self.sock.listen(32)
        self.port = self.sock.getsockname()[1]
        self.commands: list[str] = []
        self._lock = threading.Lock()
        self._stop = False
        self._conns: list[socket.socket] = []
        threading.Thread(target=self._accept, daemon=True).start()

    @property
    def url(self) -> str:
        return f"mongodb://127.0.0.1:{self.port}/?directConnection=true&serverSelectionTimeoutMS=5000"

    def close(self):
        self._stop = True
        for c in list(self._conns):
            try:
                c.close()
            except OSError:
                pass
        self.sock.close()

    # ---- framing ----
    def _accept(self):
        while not self._stop:
            try:
                conn, _ = self.sock.accept()
            except OSError:
                return
            self._conns.append(conn)
            threading.Thread(target=self._serve, args=(conn,), daemon=True).start()

    @staticmethod
    def _recv(conn, n):
        buf = b""
        while len(buf) < n:
            chunk = conn.recv(n - len(buf))
            if not chunk:
                raise ConnectionError
            buf += chunk
        return buf

    def _serve(self, conn):
        try:
            while not self._stop:
                length, req_id, _, op = struct.unpack("<iiii", self._recv(conn, 16))
                body = self._recv(conn, length - 16)
                if op == OP_QUERY:
                    _flags, = struct.unpack_from("<i", body, 0)
                    end = body.index(b"\x00", 4)
                    cmd = bson.decode(body[end + 9:end + 9 + struct.unpack_from("<i", body, end + 9)[0]], _CODEC)
                    reply = bson.encode(self._dispatch(cmd))
                    payload = struct.pack("<iqii", 0, 0, 0, 1) + reply
                    conn.sendall(struct.pack("<iiii", 16 + len(payload), req_id, req_id, OP_REPLY) + payload)
                elif op == OP_MSG:
                    flags, = struct.unpack_from("<I", body, 0)
                    pos, end = 4, len(body) - (4 if flags & 1 else 0)
                    cmd = None
                    seqs = {}
                    while pos < end:
                        kind = body[pos]
                        pos += 1
                        if kind == 0:
                            n, = struct.unpack_from("<i", body, pos)
                            cmd = bson.decode(body[pos:pos + n], _CODEC)
                            pos += n
                        else:
                            size, = struct.unpack_from("<i", body, pos)
                            sec = body[pos + 4:pos + size]
                            ident_end = sec.index(b"\x00")
                            ident = sec[:ident_end].decode()
                            seqs[ident] = bson.decode_all(sec[ident_end + 1:], _CODEC)
                            pos += size
                    cmd.update(seqs)
                    reply = bson.encode(self._dispatch(cmd))
                    payload = struct.pack("<I", 0) + b"\x00" + reply
                    conn.sendall(struct.pack("<iiii", 16 + len(payload), req_id, req_id, OP_MSG) + payload)
                else:
                    raise ConnectionError(f"unsupported opcode {op}")
        except (ConnectionError, OSError):
            pass
        finally:
            try:
                conn.close()
            except OSError:
                pass

    # ---- commands ----
    def _dispatch(self, cmd: dict) -> dict:
        name = next(iter(cmd))
        with self._lock:
            self.commands.append(name)
            try:
                out = self.loop.run_until_complete(self._command(name, cmd))
            except Exception as e:  # noqa: BLE001 -- reported like a server error
                return {"ok": 0, "errmsg": f"{type(e).__name__}: {e}", "code": 2}
        out.setdefault("ok", 1)
        return out

    async def _command(self, name: str, cmd: dict) -> dict:
        lname = name.lower()
        if lname in ("hello", "ismaster"):
            return {"helloOk": True, "isWritablePrimary": True, "ismaster": True, "maxBsonObjectSize": 16 * 1024 * 1024,
                    "maxMessageSizeBytes": 48_000_000, "maxWriteBatchSize": 100_000,
                    "localTime": dt.datetime.now(dt.timezone.utc), "logicalSessionTimeoutMinutes": 30,
                    "connectionId": 1, "minWireVersion": 0, "maxWireVersion": 21, "readOnly": False}
        if lname in ("ping", "endsessions", "killcursors"):
            return {}
        if lname == "buildinfo":
            return {"version": "7.0.0", "versionArray": [7, 0, 0, 0]}
        db = self.client[cmd.get("$db", "test")]
        coll = db[cmd[name]] if isinstance(cmd[name], str) else None
        ns = f"{cmd.get('$db', 'test')}.{cmd[name]}"
        if lname == "createindexes":
            for ix in cmd["indexes"]:
                keys = list(ix["key"].items())
                await coll.create_index(keys[0][0] if len(keys) == 1 else keys, unique=bool(ix.get("unique")))
            return {"numIndexesBefore": 1, "numIndexesAfter": 1 + len(cmd["indexes"])}
        if lname == "insert":
            n, errors = 0, []
            for i, d in enumerate(cmd["documents"]):
                try:
                    await coll.insert_one(d)
                    n += 1
                except DuplicateKeyError as e:
                    errors.append({"index": i, "code": 11000, "errmsg": f"E11000 duplicate key error: {e}"})
                    if cmd.get("ordered", True):
                        break
            return {"n": n, **({"writeErrors": errors} if errors else {})}
        if lname == "update":
            n = nmod = 0
            upserted = []
            for i, u in enumerate(cmd["updates"]):
                if u.get("multi"):
                    r = await coll.update_many(u["q"], u["u"])
                else:
                    r = await coll.update_one(u["q"], u["u"], upsert=bool(u.get("upsert")))
                n += r.matched_count
                nmod += r.modified_count
                if getattr(r, "upserted_id", None) is not None:
                    upserted.append({"index": i, "_id": r.upserted_id})
                    n += 1
            return {"n": n, "nModified": nmod, **({"upserted": upserted} if upserted else {})}
        if lname == "delete":
            n = 0
            for d in cmd["deletes"]:
                r = await (coll.delete_one(d["q"]) if d.get("limit", 0) == 1 else coll.delete_many(d["q"]))
                n += r.deleted_count
            return {"n": n}
        if lname == "find":
            docs = await coll.find(cmd.get("filter") or {}).to_list(length=None)
            for key, direction in reversed(list((cmd.get("sort") or {}).items())):
                docs.sort(key=lambda d: (d.get(key) is None, d.get(key)), reverse=direction < 0)
            docs = docs[cmd.get("skip", 0):]
            if cmd.get("limit"):
                docs = docs[:abs(cmd["limit"])]
            proj = cmd.get("projection")
            if proj and all(v in (1, True) for k, v in proj.items() if k != "_id"):
                keep = {k for k, v in proj.items() if v}
                docs = [{k: v for k, v in d.items() if k in keep or (k == "_id" and proj.get("_id", 1))} for d in docs]
            return {"cursor": {"firstBatch": docs, "id": 0, "ns": ns}}
        if lname == "aggregate":
            docs = await coll.aggregate(cmd["pipeline"]).to_list(length=None)
            return {"cursor": {"firstBatch": docs, "id": 0, "ns": ns}}
        if lname == "getmore":
            return {"cursor": {"nextBatch": [], "id": 0, "ns": ns}}
        raise NotImplementedError(f"command {name}")
