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

Pinning: the char leaves of PartialMerkleTreeTest.kt:22-25 are the derived fixture
(tests/golden/merkle_vectors.json "ref_*"); the Ed25519 key leaf (class id 45 +
writeBytesWithLength) is pinned by the reference's own serialised keys
(tests/golden/kryo_key_vectors.json, samples/irs-demo/.../trade.json:3,25); every
other kind -- Party, the issue Command -- is PARITY UNPINNED (no Kryo, no JVM
here: the bytes follow the published format, unconfirmed).
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


def chunked(data: bytes) -> bytes:
    """OutputChunked(output, 1024) + endChunks(): <= 1024-byte chunks, each after
    its varint length, then a zero-length chunk (CompatibleFieldSerializer's
    per-field framing)."""
    out = bytearray()
    for p in range(0, len(data), 1024):
        c = data[p:p + 1024]
        out += varint(len(c)) + c
    return bytes(out) + b"\x00"


def class_name(name_id: int, name: str) -> bytes:
    """DefaultClassResolver.writeName: NAME + 2 (= 1), the graph's name id, the name."""
    return varint(1) + varint(name_id) + write_string(name)


def fields_header(names) -> bytes:
    """CompatibleFieldSerializer's first write of a class in a graph: the field
    count and the EXTENDED cached names ("DeclaringSimpleName.field"), sorted."""
    names = sorted(names)
    return varint(len(names)) + b"".join(write_string(n) for n in names)


def key_value(key_class: int, key: bytes) -> bytes:
    """A key whose concrete class the field does not fix: class + writeBytesWithLength."""
    return varint(key_class + 2) + varint(len(key)) + bytes(key)


def party_body(name_der: bytes, key: bytes, key_class: int, x500_class: int) -> bytes:
    """net.corda.core.identity.Party (identity/Party.kt: name: X500Name,
    AbstractParty.owningKey: PublicKey) through CompatibleFieldSerializer; the
    name via X500NameSerializer (Kryo.kt:615-624: writeBytes(encoded))."""
    return (class_name(0, "net.corda.core.identity.Party") + fields_header(["AbstractParty.owningKey", "Party.name"])
            + chunked(key_value(key_class, key)) + chunked(varint(x500_class + 2) + bytes(name_der)))


def issue_command_body(cls: str, nonce: int, keys, aal_class: int) -> bytes:
    """Command(value = <cls>(nonce: Long), signers = Arrays.asList(PublicKey[]))
    (Structures.kt:285, TransactionBuilder.kt:124, Cash.kt:148): fields sorted
    Command.signers, Command.value; the list via ArraysAsListSerializer
    (kryo-serializers 0.41: length, component class, elements); PublicKey and the
    command class by implicit NAME registration (name ids 1, 2)."""
    signers = (varint(aal_class + 2) + varint(len(keys)) + class_name(1, "java.security.PublicKey")
               + b"".join(key_value(kc, k) for kc, k in keys))
    simple = cls.replace("$", ".").rsplit(".", 1)[-1]
    value = class_name(2, cls) + fields_header([simple + ".nonce"]) + chunked(varlong_zigzag(nonce))
    return (class_name(0, "net.corda.core.contracts.Command") + fields_header(["Command.signers", "Command.value"])
            + chunked(signers) + chunked(value))


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
        "party": lambda: party_body(value[0], value[1], value[2], class_id),
        "issue_command": lambda: issue_command_body(value[0], value[1], value[2], class_id),
    }[kind]
    return HEADER + body()


TRANSACTION_TYPE_GENERAL = "net.corda.core.contracts.TransactionType$General"  # TransactionTypes.kt:64
