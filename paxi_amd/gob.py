"""The encoding/gob wire format, restated for the messages Paxi sends between
replicas over its TCP transport.

The reference's transport writes every message with one `gob.Encoder` per
connection, `encoder.Encode(&m)` on an `interface{}` (transport.go:108-116),
and reads it back with one `gob.Decoder` per accepted connection,
`decoder.Decode(&m)` (transport.go:146-165).  The concrete types travel under
the names `gob.Register` gives them (message.go:8-17, paxos/msg.go:10-16,
abd/msg.go:9-14, wpaxos/msg.go:11-18).

encoding/gob is Go's standard library, absent from this image like the rest of
Go; this is a restatement of its published format (encoding/gob doc.go,
"Encoding Details"), not of Go source:

- uint: < 128 one byte, else the byte count negated then the big-endian bytes;
  int: zig-zag (`x << 1`, or `^x << 1 | 1` when negative) as a uint;
  string / []byte: uint length then the bytes;
- a stream is a sequence of messages `uint(length) payload`; a payload opens
  with an int type id: negative = the definition of type -id (a wireType
  struct), positive = a value of that type;
- a struct value is `(uint field delta, value)*` ended by 0, zero-valued
  fields omitted (a nested struct is always sent; a nil map is omitted, an
  empty non-nil one is sent); a map is `uint count (key value)*`;
- a top-level non-struct value (here the `interface{}` the transport
  encodes) is a singleton: `0` then the value;
- an interface value is `uint(len(name)) name`, then the definitions of
  types not yet sent on this stream (the first one continues the current
  message, each later one and then the value go out as messages of their
  own), then `int(type id) uint(len) value`;
- user type ids start at 65 in a fresh process and are handed out as types
  are first built: a struct takes its id before its fields, a map or slice
  after its key / element types.  Type definitions are sent once per
  encoder (stream), on first use.

Pinned against the worked example in the encoding/gob documentation (Point
{22, 33}, tests/golden/gob_kats.json); no Go toolchain exists here to check a
Paxi stream byte for byte, so the Paxi-level streams are parity-unpinned
 and checked by round trips and the replay test.
"""
from __future__ import annotations

import io

# ---- builtin type ids (encoding/gob type.go bootstrap order) ---------------
BOOL, INT, UINT, FLOAT, BYTES, STRING, COMPLEX, INTERFACE = 1, 2, 3, 4, 5, 6, 7, 8
WIRETYPE = 16
FIRST_USER_ID = 65
_BUILTIN_NAMES = {BOOL: "bool", INT: "int", UINT: "uint", FLOAT: "float", BYTES: "bytes", STRING: "string",
                  COMPLEX: "complex", INTERFACE: "interface"}


class GobError(ValueError):
    pass


# ---- Go type model ----------------------------------------------------------
class Struct:
    def __init__(self, name, fields):
        self.name = name
        self.fields = list(fields)          # [(field name, type)]; type: builtin id or Struct/Map/Slice


class Map:
    def __init__(self, name, key, elem):
        self.name, self.key, self.elem = name, key, elem


class Slice:
    def __init__(self, name, elem):
        self.name, self.elem = name, elem


# Paxi's types (db.go:10-24, message.go:24-48, ballot.go:10, id.go:11)
BALLOT, ID, KEY, VALUE = UINT, STRING, INT, BYTES
PROPERTIES = Map("map[string]string", STRING, STRING)
COMMAND = Struct("Command", [("Key", KEY), ("Value", VALUE), ("ClientID", ID), ("CommandID", INT)])
REQUEST = Struct("Request", [("Command", COMMAND), ("Properties", PROPERTIES), ("Timestamp", INT), ("NodeID", ID)])
REPLY = Struct("Reply", [("Command", COMMAND), ("Value", VALUE), ("Properties", PROPERTIES), ("Timestamp", INT),
                         ("Err", INTERFACE)])
# paxos/msg.go:19-70
P1A = Struct("P1a", [("Ballot", BALLOT)])
COMMAND_BALLOT = Struct("CommandBallot", [("Command", COMMAND), ("Ballot", BALLOT)])
P1B = Struct("P1b", [("Ballot", BALLOT), ("ID", ID), ("Log", Map("map[int]paxos.CommandBallot", INT, COMMAND_BALLOT))])
P2A = Struct("P2a", [("Ballot", BALLOT), ("Slot", INT), ("Command", COMMAND)])
P2B = Struct("P2b", [("Ballot", BALLOT), ("ID", ID), ("Slot", INT)])
P3 = Struct("P3", [("Ballot", BALLOT), ("Slot", INT), ("Command", COMMAND)])
# abd/msg.go:16-46
ABD_GET = Struct("Get", [("ID", ID), ("CID", INT), ("Key", KEY)])
ABD_GETREPLY = Struct("GetReply", [("ID", ID), ("CID", INT), ("Key", KEY), ("Value", VALUE), ("Version", INT)])
ABD_SET = Struct("Set", [("ID", ID), ("CID", INT), ("Key", KEY), ("Value", VALUE), ("Version", INT)])
ABD_SETREPLY = Struct("SetReply", [("ID", ID), ("CID", INT), ("Key", KEY)])
# wpaxos/msg.go:22-84, m2paxos/msg.go:25-80, kpaxos/msg.go:25-80: one set of
# per-key wrappers per package (distinct Go types of the same shape); the
# embedded paxos message is a field named after its type
def _keyed():
    return {"Prepare": Struct("Prepare", [("Key", KEY), ("P1a", P1A)]),
            "Promise": Struct("Promise", [("Key", KEY), ("P1b", P1B)]),
            "Accept": Struct("Accept", [("Key", KEY), ("P2a", P2A)]),
            "Accepted": Struct("Accepted", [("Key", KEY), ("P2b", P2B)]),
            "Commit": Struct("Commit", [("Key", KEY), ("P3", P3)]),
            "LeaderChange": Struct("LeaderChange", [("Key", KEY), ("To", ID), ("From", ID), ("Ballot", BALLOT)])}


KEYED = {pkg: _keyed() for pkg in ("wpaxos", "m2paxos", "kpaxos")}
# epaxos/msg.go:18-65: instance messages with dependency maps
DEPS = Map("map[paxi.ID]int", ID, INT)
EP_PREACCEPT = Struct("PreAccept", [("Ballot", BALLOT), ("Replica", ID), ("Slot", INT), ("Command", COMMAND),
                                    ("Seq", INT), ("Dep", DEPS)])
EP_PREACCEPTREPLY = Struct("PreAcceptReply", [("Ballot", BALLOT), ("Replica", ID), ("Slot", INT), ("Seq", INT),
                                              ("Dep", DEPS), ("Committed", DEPS)])
EP_ACCEPT = Struct("Accept", [("Ballot", BALLOT), ("Replica", ID), ("Slot", INT), ("Seq", INT), ("Dep", DEPS)])
EP_ACCEPTREPLY = Struct("AcceptReply", [("Ballot", BALLOT), ("Replica", ID), ("Slot", INT)])
EP_COMMIT = Struct("Commit", [("Ballot", BALLOT), ("Replica", ID), ("Slot", INT), ("Command", COMMAND),
                              ("Seq", INT), ("Dep", DEPS)])
WP_PREPARE, WP_PROMISE, WP_ACCEPT = KEYED["wpaxos"]["Prepare"], KEYED["wpaxos"]["Promise"], KEYED["wpaxos"]["Accept"]
WP_ACCEPTED, WP_COMMIT = KEYED["wpaxos"]["Accepted"], KEYED["wpaxos"]["Commit"]
WP_LEADERCHANGE = KEYED["wpaxos"]["LeaderChange"]

# gob.Register names: the package path "." the type name (the reference builds
# under the GOPATH import path github.com/ailidani/paxi)
PKG = "github.com/ailidani/paxi"
REGISTERED = {
    f"{PKG}.Request": REQUEST, f"{PKG}.Reply": REPLY,
    f"{PKG}/paxos.P1a": P1A, f"{PKG}/paxos.P1b": P1B, f"{PKG}/paxos.P2a": P2A, f"{PKG}/paxos.P2b": P2B,
    f"{PKG}/paxos.P3": P3,
    f"{PKG}/abd.Get": ABD_GET, f"{PKG}/abd.GetReply": ABD_GETREPLY, f"{PKG}/abd.Set": ABD_SET,
    f"{PKG}/abd.SetReply": ABD_SETREPLY,
}
REGISTERED.update({f"{PKG}/{pkg}.{name}": t for pkg, types in KEYED.items() for name, t in types.items()})
REGISTERED.update({f"{PKG}/epaxos.PreAccept": EP_PREACCEPT, f"{PKG}/epaxos.PreAcceptReply": EP_PREACCEPTREPLY,
                   f"{PKG}/epaxos.Accept": EP_ACCEPT, f"{PKG}/epaxos.AcceptReply": EP_ACCEPTREPLY,
                   f"{PKG}/epaxos.Commit": EP_COMMIT})


# ---- primitives -------------------------------------------------------------
def enc_uint(x: int) -> bytes:
    if x < 0:
        raise GobError("negative uint")
    if x < 128:
        return bytes([x])
    b = x.to_bytes((x.bit_length() + 7) // 8, "big")
    return bytes([256 - len(b)]) + b


def enc_int(x: int) -> bytes:
    return enc_uint((~x << 1) | 1 if x < 0 else x << 1)


def enc_bytes(b: bytes) -> bytes:
    return enc_uint(len(b)) + bytes(b)


class Reader:
    def __init__(self, data: bytes):
        self.b = memoryview(bytes(data))
        self.i = 0

    def left(self):
        return len(self.b) - self.i

    def byte(self):
        if self.i >= len(self.b):
            raise GobError("unexpected end of data")
        v = self.b[self.i]
        self.i += 1
        return v

    def take(self, n):
        if n > self.left():
            raise GobError("unexpected end of data")
        v = bytes(self.b[self.i:self.i + n])
        self.i += n
        return v

    def uint(self):
        c = self.byte()
        if c < 128:
            return c
        n = 256 - c
        if n > 8:
            raise GobError("uint too long")
        return int.from_bytes(self.take(n), "big")

    def int(self):
        u = self.uint()
        return ~(u >> 1) if u & 1 else u >> 1


def _float(u: int) -> float:
    import struct
    return struct.unpack("<d", u.to_bytes(8, "big"))[0]   # the uint holds the bytes in reverse order


def enc_float(x: float) -> bytes:
    import struct
    return enc_uint(int.from_bytes(struct.pack("<d", x), "big"))


# ---- type registry: ids as a fresh Go process hands them out ----------------
class TypeIds:
    """Process-global type ids (encoding/gob type.go: nextId).  One instance
    plays one Go process: every encoder (stream) it serves shares the ids."""

    def __init__(self):
        self.next = FIRST_USER_ID
        self.ids = {}                     # id(type object) -> type id
        self.wire = {}                    # type id -> (type object, field ids)

    def id_of(self, t):
        if isinstance(t, int):
            return t
        k = id(t)
        if k in self.ids:
            return self.ids[k]
        if isinstance(t, Struct):         # newStructType sets the id before the fields are built
            tid = self._take(t)
            fids = [self.id_of(ft) for _, ft in t.fields]
            self.wire[tid] = (t, fids)
            return tid
        if isinstance(t, Map):            # mapType.init: after key and element
            kid, eid = self.id_of(t.key), self.id_of(t.elem)
            tid = self._take(t)
            self.wire[tid] = (t, [kid, eid])
            return tid
        if isinstance(t, Slice):
            eid = self.id_of(t.elem)
            tid = self._take(t)
            self.wire[tid] = (t, [eid])
            return tid
        raise GobError(f"not a gob type: {t!r}")

    def _take(self, t):
        tid = self.next
        self.next += 1
        self.ids[id(t)] = tid
        return tid


def _wire_type(t, tid, fids) -> bytes:
    """encodingOfWireType: wireType{ArrayT, SliceT, StructT, MapT, ...} with one field set."""
    common = enc_uint(1) + enc_bytes(t.name.encode()) + enc_uint(1) + enc_int(tid) + enc_uint(0)   # CommonType
    if isinstance(t, Struct):
        body = enc_uint(1) + common                                    # structType.CommonType
        if t.fields:
            body += enc_uint(1) + enc_uint(len(t.fields))              # structType.Field []*fieldType
            for (fname, _), fid in zip(t.fields, fids):
                body += enc_uint(1) + enc_bytes(fname.encode()) + enc_uint(1) + enc_int(fid) + enc_uint(0)
        return enc_uint(3) + body + enc_uint(0) + enc_uint(0)         # wireType.StructT (field 2)
    if isinstance(t, Map):
        body = enc_uint(1) + common + enc_uint(1) + enc_int(fids[0]) + enc_uint(1) + enc_int(fids[1])
        return enc_uint(4) + body + enc_uint(0) + enc_uint(0)         # wireType.MapT (field 3)
    body = enc_uint(1) + common + enc_uint(1) + enc_int(fids[0])
    return enc_uint(2) + body + enc_uint(0) + enc_uint(0)             # wireType.SliceT (field 1)


# ---- encoder ------------------------------------------------------------------
def _zero(t, v):
    if v is None:
        return True
    if isinstance(t, int):
        return t in (INT, UINT, BOOL, FLOAT, COMPLEX) and v == 0 or t in (STRING, BYTES) and len(v) == 0
    if isinstance(t, Slice):
        return len(v) == 0
    return False   # structs are always sent, an empty non-nil map too


def _enc_value(t, v, reg: TypeIds) -> bytes:
    if isinstance(t, int):
        if t in (INT,):
            return enc_int(int(v))
        if t in (UINT, BOOL):
            return enc_uint(int(v))
        if t == STRING:
            return enc_bytes(v.encode() if isinstance(v, str) else v)
        if t == BYTES:
            return enc_bytes(v)
        if t == FLOAT:
            return enc_float(float(v))
        if t == COMPLEX:                                   # real part, then imaginary
            return enc_float(complex(v).real) + enc_float(complex(v).imag)
        if t == INTERFACE:
            raise GobError("only nil interface fields are encoded here")
        raise GobError(f"builtin {t} not supported")
    if isinstance(t, Struct):
        out = b""
        last = -1
        for i, (fname, ft) in enumerate(t.fields):
            fv = v.get(fname) if isinstance(v, dict) else None
            if ft == INTERFACE or _zero(ft, fv) and not isinstance(ft, Struct):
                continue
            if isinstance(ft, Struct) and fv is None:
                fv = {}
            out += enc_uint(i - last) + _enc_value(ft, fv, reg)
            last = i
        return out + enc_uint(0)
    if isinstance(t, Map):
        items = sorted(v.items())        # Go's map order is random; any order decodes the same
        out = enc_uint(len(items))
        for k, e in items:
            out += _enc_value(t.key, k, reg) + _enc_value(t.elem, e, reg)
        return out
    if isinstance(t, Slice):
        out = enc_uint(len(v))
        for e in v:
            out += _enc_value(t.elem, e, reg)
        return out
    raise GobError(f"bad type {t!r}")


class Encoder:
    """One gob.Encoder: a connection's stream (transport.go:108)."""

    def __init__(self, reg: TypeIds | None = None):
        self.reg = reg or TypeIds()
        self.sent = set()
        self.out = io.BytesIO()

    def _defs(self, t, acc):
        """sendType order: a type's definition, then (recursively) its fields' types."""
        if isinstance(t, int):
            return
        tid = self.reg.id_of(t)
        if tid in self.sent:
            return
        self.sent.add(tid)
        acc.append(enc_int(-tid) + _wire_type(t, tid, self.reg.wire[tid][1]))
        inner = [ft for _, ft in t.fields] if isinstance(t, Struct) else \
            [t.key, t.elem] if isinstance(t, Map) else [t.elem]
        for ft in inner:
            self._defs(ft, acc)

    def encode_interface(self, name: str, value) -> bytes:
        """Encode(&m) with m an interface{} holding `value` of registered type `name`."""
        t = REGISTERED.get(name)
        if t is None:
            raise GobError(f"type not registered for interface: {name}")
        head = enc_int(INTERFACE) + enc_uint(0) + enc_bytes(name.encode())   # singleton delta 0, then the name
        defs = []
        self._defs(t, defs)
        body = _enc_value(t, value, self.reg)
        tail = enc_int(self.reg.id_of(t)) + enc_uint(len(body)) + body
        msgs = []
        if defs:
            msgs.append(head + defs[0])
            msgs.extend(defs[1:])
            msgs.append(tail)
        else:
            msgs.append(head + tail)
        data = b"".join(enc_uint(len(m)) + m for m in msgs)
        self.out.write(data)
        return data

    def getvalue(self) -> bytes:
        return self.out.getvalue()


# ---- decoder ------------------------------------------------------------------
class Decoder:
    """One gob.Decoder over a whole stream: decode() returns (name, value) per
    Encode of an interface{} (transport.go:146-165).  Types come from the
    stream's own definitions; values are dicts of the fields sent, with the
    omitted (zero) ones filled in."""

    def __init__(self, data: bytes):
        self.r = Reader(data)
        self.types = {}          # id -> ("struct", name, [(fname, id)]) | ("map", name, kid, eid) | ("slice", name, eid)
        self.msg = None          # Reader over the current message

    def _next_msg(self):
        if self.r.left() == 0:
            return False
        n = self.r.uint()
        self.msg = Reader(self.r.take(n))
        return True

    def _wire(self, m: Reader):
        """Decode an encodingOfWireType."""
        def common(m):
            name, tid = "", 0
            f = -1
            while True:
                d = m.uint()
                if d == 0:
                    return name, tid
                f += d
                if f == 0:
                    name = m.take(m.uint()).decode()
                elif f == 1:
                    tid = m.int()
                else:
                    raise GobError("bad CommonType")
        f = -1
        out = None
        while True:
            d = m.uint()
            if d == 0:
                break
            f += d
            sf = -1
            name, tid, fields, key, elem = "", 0, [], 0, 0
            while True:
                dd = m.uint()
                if dd == 0:
                    break
                sf += dd
                if sf == 0:
                    name, tid = common(m)
                elif f == 2 and sf == 1:                 # structType.Field
                    for _ in range(m.uint()):
                        fname, fid, ff = "", 0, -1
                        while True:
                            d3 = m.uint()
                            if d3 == 0:
                                break
                            ff += d3
                            if ff == 0:
                                fname = m.take(m.uint()).decode()
                            elif ff == 1:
                                fid = m.int()
                        fields.append((fname, fid))
                elif f == 3 and sf == 1:
                    key = m.int()
                elif f == 3 and sf == 2:
                    elem = m.int()
                elif f in (0, 1) and sf == 1:
                    elem = m.int()
                elif f == 0 and sf == 2:
                    m.int()                               # array length
                else:
                    raise GobError(f"unsupported wireType field {f}.{sf}")
            if f == 2:
                out = ("struct", name, fields)
            elif f == 3:
                out = ("map", name, key, elem)
            elif f in (0, 1):
                out = ("slice", name, elem)
            else:
                raise GobError(f"unsupported wireType {f}")
        if out is None:
            raise GobError("empty wireType")
        return out

    def _type_sequence(self, m: Reader, interface: bool):
        """decodeTypeSequence: definitions, then the id of the value that follows."""
        while True:
            if m.left() == 0:
                if not self._next_msg():
                    raise GobError("unexpected end of stream")
                m = self.msg
            tid = m.int()
            if tid >= 0:
                return tid, m
            self.types[-tid] = self._wire(m)
            if m.left() > 0:
                if not interface:
                    raise GobError("extra data in buffer")
                m.uint()                                  # a delimited definition follows in-line

    def _zero_of(self, tid):
        if tid in (INT, UINT):
            return 0
        if tid == BOOL:
            return False
        if tid == STRING:
            return ""
        if tid == FLOAT:                                  # Go's 0.0 and 0i for an omitted field
            return 0.0
        if tid == COMPLEX:
            return 0j
        if tid == BYTES:
            return None
        if tid == INTERFACE:
            return None
        t = self.types.get(tid)
        if t and t[0] == "struct":
            return {fn: self._zero_of(fid) for fn, fid in t[2]}
        return None

    def _value(self, tid, m: Reader):
        if tid == INT:
            return m.int()
        if tid in (UINT,):
            return m.uint()
        if tid == BOOL:
            return m.uint() != 0
        if tid == FLOAT:                                  # float64 bits, byte-reversed, as a uint
            return _float(m.uint())
        if tid == COMPLEX:
            re = _float(m.uint())
            return complex(re, _float(m.uint()))
        if tid == STRING:
            return m.take(m.uint()).decode()
        if tid == BYTES:
            return m.take(m.uint())
        if tid == INTERFACE:
            return self._interface(m)
        t = self.types.get(tid)
        if t is None:
            raise GobError(f"unknown type id {tid}")
        if t[0] == "struct":
            v = {fn: self._zero_of(fid) for fn, fid in t[2]}
            f = -1
            while True:
                d = m.uint()
                if d == 0:
                    return v
                f += d
                if f >= len(t[2]):
                    raise GobError("field number out of range")
                fn, fid = t[2][f]
                v[fn] = self._value(fid, m)
        if t[0] == "map":
            return {self._value(t[2], m): self._value(t[3], m) for _ in range(m.uint())}
        return [self._value(t[2], m) for _ in range(m.uint())]

    def _interface(self, m: Reader):
        n = m.uint()
        if n == 0:
            return None                                   # nil interface
        name = m.take(n).decode()
        tid, m2 = self._type_sequence(m, True)
        ln = m2.uint()
        body = Reader(m2.take(ln))
        return name, self._value(tid, body)

    def decode(self):
        """The next Encode(&m) of the stream as (registered name, value), or None at its end."""
        if not self._next_msg():
            return None
        tid, m = self._type_sequence(self.msg, False)
        if tid != INTERFACE:
            raise GobError(f"top-level value of type {tid}, not interface{{}}")
        if m.uint() != 0:
            raise GobError("non-zero delta for singleton")
        v = self._interface(m)
        return v

    def __iter__(self):
        while True:
            v = self.decode()
            if v is None:
                return
            yield v


def full(t, v):
    """v with every omitted field set to its zero value, as the decoder returns it."""
    if isinstance(t, Struct):
        v = v or {}
        return {fn: full(ft, v.get(fn)) for fn, ft in t.fields}
    if isinstance(t, Map):
        return None if v is None else {k: full(t.elem, e) for k, e in v.items()}
    if isinstance(t, Slice):
        return [full(t.elem, e) for e in v or []]
    if v is None:
        zero = {INT: 0, UINT: 0, STRING: "", BOOL: False, FLOAT: 0.0, COMPLEX: 0j}
        return zero.get(t) if isinstance(t, int) else None
    if t == BYTES and len(v) == 0:
        return None
    return v


# ---- the documentation's worked example (tests/golden/gob_kats.json) --------
def encode_point_example(x: int, y: int) -> bytes:
    """enc.Encode(Point{X, Y}) for `type Point struct {X, Y int}` in a fresh
    process: the type definition message, then the value message."""
    reg = TypeIds()
    pt = Struct("Point", [("X", INT), ("Y", INT)])
    tid = reg.id_of(pt)
    d = enc_int(-tid) + _wire_type(pt, tid, reg.wire[tid][1])
    v = enc_int(tid) + _enc_value(pt, {"X": x, "Y": y}, reg)
    return enc_uint(len(d)) + d + enc_uint(len(v)) + v
