"""Kryo leaf preimages (TEST INFRASTRUCTURE ONLY: the checker of
corda_amd/csrc/kryo.cpp; the product never imports oracle/).

Restates, for the component kinds cordahip_kryo_encode supports, what
serializedHash (core/.../transactions/MerkleTransaction.kt:16-18) hashes:
"corda\\0\\0\\1" (Kryo.kt:101) + Kryo.writeClassAndObject (Kryo.kt:165-176),
references off. Kryo 4.0.0 (com.esotericsoftware:kryo:4.0.0, core/build.gradle:56,
not in /root/reference) wire format, restated from its published source:
  Output.writeVarInt(v, true)   7-bit groups, low first, 0x80 = more
  Output.writeString(s)         null 0x80, "" 0x81; 2..63 ASCII chars: the bytes with
                                the last | 0x80; else writeUtf8Length(len + 1) then
                                1/2/3-byte UTF-8 per UTF-16 code unit
  writeInt/Long/Short/Char      big-endian fixed width (the boxed primitives'
                                default serializers)
  DefaultClassResolver.writeClass  registered: varint(id + 2); implicit NAME
                                registration: varint(1), varint(name id), name string
  default registrations         int 0, String 1, float 2, boolean 3, byte 4, char 5,
                                short 6, long 7, double 8, void 9
Corda serializers: Ed25519PublicKeySerializer (Kryo.kt:383-393), PublicKeySerializer
(:441-451), X500NameSerializer (:615-624), CordaClassResolver.registerImplicit's
KotlinObjectSerializer and NAME registration (CordaClassResolver.kt:76-99);
Kryo's CompatibleFieldSerializer (the default serializer, EXTENDED cached field
names: DefaultKryoCustomizer.kt:56-58) with OutputChunked field framing, and
kryo-serializers 0.41's ArraysAsListSerializer (DefaultKryoCustomizer.kt:60).

Object graphs (Party, the issue Command, TransactionState<Cash.State>) are
written by a literal model of Kryo's buffered Output classes (class Output /
OutputChunked below, method for method: require, writeBytes, flush,
writeChunkSize, endChunks), so the framing of NESTED CompatibleFieldSerializers
falls out of the same rules Kryo runs: an inner endChunks() flushes every
enclosing OutputChunked (Output.flush() flushes its stream), cutting the
enclosing field's chunk, and the inner 0 terminator opens a new one (ADVICE r03:
an issue command's value field is [len A] A [01 00] [00], not one chunk).

Pinning: the char leaves of PartialMerkleTreeTest.kt:22-25 are the derived fixture
(tests/golden/merkle_vectors.json "ref_*"); the Ed25519 key leaf (class id 45 +
writeBytesWithLength) is pinned by the reference's own serialised keys
(tests/golden/kryo_key_vectors.json, samples/irs-demo/.../trade.json:3,25); every
other kind -- Party, the issue Command, the cash TransactionState -- is PARITY
UNPINNED (no Kryo, no JVM here: the bytes follow the published format,
unconfirmed by any reference output).
"""
import struct

HEADER = b"corda\x00\x00\x01"
ID = {"int": 0, "String": 1, "float": 2, "boolean": 3, "byte": 4, "char": 5, "short": 6, "long": 7, "double": 8}


def varint(v: int) -> bytes:
    out = bytearray()
    while v >> 7:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def utf8_length(v: int) -> bytes:
    if v >> 6 == 0:
        return bytes([v | 0x80])
    groups = [(v | 0xC0) & 0xFF]
    rest = v >> 6
    shifts = [7, 7, 7, 7]
    while True:
        nxt = rest >> shifts.pop(0) if shifts else 0
        if nxt == 0:
            groups.append(rest & 0xFF)
            break
        groups.append((rest & 0x7F) | 0x80)
        rest = nxt
    return bytes(groups)


def write_string(s: str) -> bytes:
    units = s.encode("utf-16-le")
    cu = [units[i] | (units[i + 1] << 8) for i in range(0, len(units), 2)]
    n = len(cu)
    if n == 0:
        return b"\x81"
    if 1 < n < 64 and all(c <= 127 for c in cu):
        b = bytearray(cu)
        b[-1] |= 0x80
        return bytes(b)
    out = bytearray(utf8_length(n + 1))
    for c in cu:
        if c <= 0x7F:
            out.append(c)
        elif c > 0x7FF:
            out += bytes([0xE0 | (c >> 12) & 0x0F, 0x80 | (c >> 6) & 0x3F, 0x80 | c & 0x3F])
        else:
            out += bytes([0xC0 | (c >> 6) & 0x1F, 0x80 | c & 0x3F])
    return bytes(out)


def varlong_zigzag(x: int) -> bytes:
    """Output.writeVarLong(x, false): zig-zag, 7-bit groups, the 9th byte 8 bits."""
    v = ((x << 1) ^ (x >> 63)) & (2**64 - 1)
    out = bytearray()
    for _ in range(8):
        if v >> 7 == 0:
            out.append(v)
            return bytes(out)
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


class Output:
    """com.esotericsoftware.kryo.io.Output: a `capacity`-byte buffer over a stream.
    The leaf's own Output (Kryo.kt:165-176: 64 KiB over a ByteArrayOutputStream)
    flushes in order, so it is modelled unbounded (stream None)."""

    def __init__(self, stream=None, capacity=None):
        self.stream, self.capacity, self.buffer = stream, capacity, bytearray()

    def require(self, required):
        if self.capacity is None or self.capacity - len(self.buffer) >= required:
            return
        self.flush()

    def write(self, value):  # Output.write(int) / writeByte
        self.require(1)
        self.buffer.append(value & 0xFF)

    def write_atomic(self, data):  # writeVarInt / writeVarLong / fixed-width: require(n), then the bytes
        self.require(len(data))
        self.buffer += data

    def write_bytes(self, data):  # Output.writeBytes: fill the buffer, flush, continue
        data = bytes(data)
        if self.capacity is None:
            self.buffer += data
            return
        count, offset = len(data), 0
        copy = min(self.capacity - len(self.buffer), count)
        while True:
            self.buffer += data[offset:offset + copy]
            count -= copy
            if count == 0:
                return
            offset += copy
            copy = min(self.capacity, count)
            self.require(copy)

    def write_string(self, s):  # Output.writeString (Java String = UTF-16 code units)
        units = s.encode("utf-16-le")
        cu = [units[i] | (units[i + 1] << 8) for i in range(0, len(units), 2)]
        n = len(cu)
        if n == 0:
            self.write(0x81)
            return
        if 1 < n < 64 and all(c <= 127 for c in cu):
            self.write_bytes(bytes(cu))  # fits: one copy; else writeAscii_slow fills piecewise
            self.buffer[-1] |= 0x80
            return
        self.write_atomic(utf8_length(n + 1))
        i = 0
        if self.capacity is None or self.capacity - len(self.buffer) >= n:
            while i < n and cu[i] <= 127:
                self.buffer.append(cu[i])
                i += 1
        while i < n:  # writeString_slow
            if self.capacity is not None and len(self.buffer) == self.capacity:
                self.require(min(self.capacity, n - i))
            c = cu[i]
            if c <= 0x7F:
                self.buffer.append(c)
            elif c > 0x7FF:
                self.buffer.append(0xE0 | (c >> 12) & 0x0F)
                self.require(2)
                self.buffer += bytes([0x80 | (c >> 6) & 0x3F, 0x80 | c & 0x3F])
            else:
                self.buffer.append(0xC0 | (c >> 6) & 0x1F)
                self.require(1)
                self.buffer.append(0x80 | c & 0x3F)
            i += 1

    def flush(self):  # Output.flush: the buffer to the stream, then stream.flush()
        if self.stream is None:
            return
        data = bytes(self.buffer)
        self.stream.write_bytes(data)
        self.stream.flush()
        self.buffer.clear()


class OutputChunked(Output):
    """com.esotericsoftware.kryo.io.OutputChunked(stream, 1024)."""

    def __init__(self, stream, size=1024):
        super().__init__(stream, size)

    def flush(self):
        if len(self.buffer) > 0:
            for b in varint(len(self.buffer)):  # writeChunkSize: stream.write(int) per byte
                self.stream.write(b)
            Output.flush(self)
        Output.flush(self)

    def end_chunks(self):
        self.flush()
        self.stream.write(0)  # the zero-length chunk


class Graph:
    """One Kryo.writeClassAndObject object graph: DefaultClassResolver's name ids and
    CompatibleFieldSerializer's header marks (graph context), both reset per leaf."""

    def __init__(self):
        self.name_ids, self.headers = {}, set()

    @staticmethod
    def write_class_id(out, reg_id):  # DefaultClassResolver.writeClass, registered
        out.write_atomic(varint(reg_id + 2))

    def write_class_name(self, out, name):  # DefaultClassResolver.writeName
        out.write_atomic(varint(1))  # NAME + 2
        if name in self.name_ids:
            out.write_atomic(varint(self.name_ids[name]))
            return
        self.name_ids[name] = len(self.name_ids)
        out.write_atomic(varint(self.name_ids[name]))
        out.write_string(name)

    def compatible_fields(self, out, cls, fields):
        """CompatibleFieldSerializer.write: fields = [(EXTENDED name, writer(output))]."""
        fields = sorted(fields, key=lambda f: f[0])
        if cls not in self.headers:
            self.headers.add(cls)
            out.write_atomic(varint(len(fields)))
            for name, _ in fields:
                out.write_string(name)
        chunked = OutputChunked(out, 1024)
        for _, w in fields:
            w(chunked)
            chunked.end_chunks()


def _leaf(write) -> bytes:
    out = Output()
    out.write_bytes(HEADER)
    write(out, Graph())
    return bytes(out.buffer)


def write_key(out, key_class, key):
    """A PublicKey of unknown concrete class: class id + writeBytesWithLength (Kryo.kt:305-308)."""
    Graph.write_class_id(out, key_class)
    out.write_atomic(varint(len(key)))
    out.write_bytes(key)


def write_party(out, g, party, x500_class, with_class=True):
    """Party (name, owningKey) or, with an empty name, AnonymousParty(owningKey)
    (identity/Party.kt, AnonymousParty.kt, AbstractParty.kt); the name through
    X500NameSerializer (Kryo.kt:615-624: writeBytes(encoded))."""
    name, key, key_class = party
    cls = "net.corda.core.identity.Party" if name else "net.corda.core.identity.AnonymousParty"
    if with_class:
        g.write_class_name(out, cls)
    fields = [("AbstractParty.owningKey", lambda o: write_key(o, key_class, key))]
    if name:
        fields.append(("Party.name", lambda o: (Graph.write_class_id(o, x500_class), o.write_bytes(name))))
    g.compatible_fields(out, cls, fields)


def write_opaque(out, g, cls, data):
    """OpaqueBytes / SecureHash$SHA256: field OpaqueBytes.bytes, byte[] (final, accepts null)."""
    g.write_class_name(out, cls)
    g.compatible_fields(out, cls, [("OpaqueBytes.bytes",
                                    lambda o: (o.write_atomic(varint(len(data) + 1)), o.write_bytes(data)))])


def leaf(kind: str, value=None, class_id: int = 0) -> bytes:
    """The serialised leaf of one component (header included)."""
    if kind == "raw":
        return bytes(value)
    body = {
        "char": lambda: varint(ID["char"] + 2) + struct.pack(">H", ord(value) if isinstance(value, str) else value),
        "short": lambda: varint(ID["short"] + 2) + struct.pack(">h", value),
        "int": lambda: varint(ID["int"] + 2) + struct.pack(">i", value),
        "long": lambda: varint(ID["long"] + 2) + struct.pack(">q", value),
        "byte": lambda: varint(ID["byte"] + 2) + struct.pack(">b", value),
        "boolean": lambda: varint(ID["boolean"] + 2) + bytes([1 if value else 0]),
        "float": lambda: varint(ID["float"] + 2) + struct.pack(">f", value),
        "double": lambda: varint(ID["double"] + 2) + struct.pack(">d", value),
        "String": lambda: varint(ID["String"] + 2) + write_string(value),
        "ed25519_key": lambda: varint(class_id + 2) + varint(32) + bytes(value),
        "public_key": lambda: varint(class_id + 2) + varint(len(value)) + bytes(value),
        "kotlin_object": lambda: varint(1) + varint(0) + write_string(value),
    }.get(kind)
    if body is not None:
        return HEADER + body()
    if kind == "party":
        return _leaf(lambda out, g: write_party(out, g, value, class_id))
    if kind == "issue_command":
        return _leaf(lambda out, g: write_issue_command(out, g, value[0], value[1], value[2], class_id))
    if kind == "cash_state":
        return _leaf(lambda out, g: write_cash_state(out, g, value, class_id))
    raise KeyError(kind)


def write_issue_command(out, g, cls, nonce, keys, aal_class):
    """Command(value = <cls>(nonce: Long), signers = Arrays.asList(PublicKey[]))
    (Structures.kt:285, TransactionBuilder.kt:124, Cash.kt:148): fields
    Command.signers, Command.value; the list via ArraysAsListSerializer
    (kryo-serializers 0.41: length, component class, elements); PublicKey and the
    command class by implicit NAME registration (name ids 1, 2); the command data's
    own CompatibleFieldSerializer nests inside the value field."""
    def signers(o):
        Graph.write_class_id(o, aal_class)
        o.write_atomic(varint(len(keys)))
        g.write_class_name(o, "java.security.PublicKey")
        for kc, k in keys:
            write_key(o, kc, k)

    simple = cls.replace("$", ".").rsplit(".", 1)[-1]

    def value(o):
        g.write_class_name(o, cls)
        g.compatible_fields(o, cls, [(simple + ".nonce", lambda c: c.write_atomic(varlong_zigzag(nonce)))])

    g.write_class_name(out, "net.corda.core.contracts.Command")
    g.compatible_fields(out, "net.corda.core.contracts.Command",
                        [("Command.signers", signers), ("Command.value", value)])


def varint_zigzag(x: int) -> bytes:
    """Output.writeVarInt(x, false) / writeInt(x, false)."""
    return varint(((x << 1) ^ (x >> 31)) & 0xFFFFFFFF)


def write_cash_state(out, g, d, x500_class):
    """TransactionState<Cash.State> of a cash issue (Cash.generateIssue, Cash.kt:166-167):
    TransactionState(data, notary, encumbrance) (Structures.kt:95-117) > Cash.State(amount,
    owner) with backing fields exitKeys = setOf(owner key, issuer key), contract =
    CASH_PROGRAM_ID, participants = listOf(owner) (Cash.kt:35,62,92-103) > Amount(quantity,
    displayTokenSize, Issued(PartyAndReference(party, reference), Currency)) (Amount.kt:37,
    Structures.kt:132,268). Final field classes (Amount, PartyAndReference, Cash, Party)
    are written NOT_NULL + body, the others class + body; BigDecimal through Kryo's
    BigDecimalSerializer (unscaled BigInteger bytes, zig-zag scale), Currency through
    CurrencySerializer (its code), LinkedHashSet through CollectionSerializer,
    Collections$SingletonList through CollectionsSingletonListSerializer."""
    issuer, owner, notary = d["issuer"], d["owner"], d["notary"]

    def amount(o):
        o.write(1)  # NOT_NULL

        def token(o3):
            g.write_class_name(o3, "net.corda.core.contracts.Issued")

            def issuer_field(o4):
                o4.write(1)
                g.compatible_fields(o4, "net.corda.core.contracts.PartyAndReference", [
                    ("PartyAndReference.party", lambda o5: write_party(o5, g, issuer, x500_class)),
                    ("PartyAndReference.reference",
                     lambda o5: write_opaque(o5, g, "net.corda.core.utilities.OpaqueBytes", d["reference"]))])

            def product(o4):
                g.write_class_name(o4, "java.util.Currency")
                o4.write_string(d["currency"])

            g.compatible_fields(o3, "net.corda.core.contracts.Issued",
                                [("Issued.issuer", issuer_field), ("Issued.product", product)])

        def display(o3):
            g.write_class_name(o3, "java.math.BigDecimal")
            unscaled = (1).to_bytes(1, "big")  # BigInteger.ONE.toByteArray()
            o3.write_atomic(varint(len(unscaled) + 1))
            o3.write_bytes(unscaled)
            o3.write_atomic(varint_zigzag(int(d["digits"])))  # scale of ONE.scaleByPowerOfTen(-digits)

        g.compatible_fields(o, "net.corda.core.contracts.Amount", [
            ("Amount.displayTokenSize", display),
            ("Amount.quantity", lambda o3: o3.write_atomic(varlong_zigzag(int(d["quantity"])))),
            ("Amount.token", token)])

    def contract(o):
        o.write(1)
        g.compatible_fields(o, "net.corda.contracts.asset.Cash", [
            ("Cash.legalContractReference",
             lambda o3: write_opaque(o3, g, "net.corda.core.crypto.SecureHash$SHA256", d["legal_ref"]))])

    def exit_keys(o):
        g.write_class_name(o, "java.util.LinkedHashSet")
        keys = []
        for _, key, kc in (owner, issuer):  # insertion order; a set
            if (kc, bytes(key)) not in keys:
                keys.append((kc, bytes(key)))
        o.write_atomic(varint(len(keys)))
        for kc, key in keys:
            write_key(o, kc, key)

    def participants(o):
        g.write_class_name(o, "java.util.Collections$SingletonList")
        write_party(o, g, owner, x500_class)

    def data(o):
        g.write_class_name(o, "net.corda.contracts.asset.Cash$State")
        g.compatible_fields(o, "net.corda.contracts.asset.Cash$State", [
            ("State.amount", amount), ("State.contract", contract), ("State.exitKeys", exit_keys),
            ("State.owner", lambda o2: write_party(o2, g, owner, x500_class)), ("State.participants", participants)])

    def encumbrance(o):
        if d.get("encumbrance") is None:
            o.write(0)  # NULL
        else:
            o.write(1)
            o.write_atomic(varint_zigzag(int(d["encumbrance"])))

    def notary_field(o):
        o.write(1)
        write_party(o, g, notary, x500_class, with_class=False)

    g.write_class_name(out, "net.corda.core.contracts.TransactionState")
    g.compatible_fields(out, "net.corda.core.contracts.TransactionState", [
        ("TransactionState.data", data), ("TransactionState.encumbrance", encumbrance),
        ("TransactionState.notary", notary_field)])


def cash_legal_ref() -> bytes:
    """Cash.legalContractReference = SecureHash.sha256(<the legal prose URL>) (Cash.kt:62)."""
    import hashlib
    return hashlib.sha256(b"https://www.big-book-of-banking-law.gov/cash-claims.html").digest()



TRANSACTION_TYPE_GENERAL = "net.corda.core.contracts.TransactionType$General"  # TransactionTypes.kt:64
