"""Hadoop-0.20 SequenceFile (v6) container and the forward index.

The device library hands out each reduce partition as a record stream in key
order (int32 recLen, int32 keyLen, TermDF bytes, ArrayListWritable bytes --
sme_index_partition_records).  This module is the host-side step after it:

  write_sequence_file    SequenceFileOutputFormat / SequenceFile.Writer [Hadoop 0.20]:
                         "SEQ\\x06", Text.writeString(key class), Text.writeString(value
                         class), compressed=0, blockCompressed=0, metadata count 0, 16-byte
                         sync; records framed as above; before a record, when
                         pos >= lastSync + 2000, int32 -1 + sync (checkAndWriteSync).
  build_forward_index    BuildIntDocVectorsForwardIndex (C/sa/edu/kaust/fwindex/
                         BuildIntDocVectorsForwardIndex.java:94-110 map, :139-153 reduce):
                         every index record in TermDF.compareTo order ->
                         writeUTF(k_gram[0] + "\\t" + (fileNo * 1e9 + pos)), where pos is the
                         reader position before the record (header end for the first).
  ForwardIndex           IntDocVectorsForwardIndex ctor + getValue(String)
                         (IntDocVectorsForwardIndex.java:93-122,148-184): term -> (file, pos)
                         -> one record read after seek.

The sync marker is random in Hadoop (MD5 of uid@time); positions do not depend
on its value, so records and the forward file are deterministic.
"""
import os
import struct

KEY_CLASS = b"sa.edu.kaust.io.TermDF"
VALUE_CLASS = b"edu.umd.cloud9.io.array.ArrayListWritable"
POSTING_CLASS = b"sa.edu.kaust.io.PostingWritable"
SYNC_ESCAPE = -1
SYNC_INTERVAL = 100 * (4 + 16)  # SequenceFile.SYNC_INTERVAL
BIG_NUMBER = 1000000000  # BuildIntDocVectorsForwardIndex.BigNumber (:113)


def _vint(n):
    """WritableUtils.writeVInt (class-name lengths are < 128: one byte)."""
    if -112 <= n <= 127:
        return struct.pack(">b", n)
    raise ValueError("vint > 127 not needed for class names")


def header(sync):
    return (b"SEQ\x06" + _vint(len(KEY_CLASS)) + KEY_CLASS + _vint(len(VALUE_CLASS)) + VALUE_CLASS
            + b"\x00\x00" + struct.pack(">i", 0) + sync)


def iter_records(buf):
    """Yield (offset, length) of each framed record of a partition stream."""
    i = 0
    while i < len(buf):
        rl = struct.unpack_from(">i", buf, i)[0]
        yield i, 8 + rl
        i += 8 + rl


def sequence_file_bytes(records, sync):
    """(file bytes, [reader position before each record])."""
    assert len(sync) == 16
    out = bytearray(header(sync))
    last_sync = 0
    positions = []
    for off, ln in iter_records(records):
        positions.append(len(out))  # SequenceFileRecordReader.getPos() before next()
        if len(out) >= last_sync + SYNC_INTERVAL and last_sync != len(out):  # checkAndWriteSync
            out += struct.pack(">i", SYNC_ESCAPE) + sync
            last_sync = len(out)
        out += records[off:off + ln]
    return bytes(out), positions


def write_sequence_file(path, records, sync=None):
    """Write one part file; returns [reader position before each record]."""
    data, positions = sequence_file_bytes(records, os.urandom(16) if sync is None else sync)
    with open(path, "wb") as f:
        f.write(data)
    return positions


def key_of(records, off):
    kl = struct.unpack_from(">i", records, off + 4)[0]
    return bytes(records[off + 8:off + 8 + kl])


def write_index_dir(ix, out_dir, sync=None):
    """The reduce output directory part-00000 .. part-(R-1) (R = the index's
    partition count).  Returns {part: [(key bytes, pos), ...]} for the forward index."""
    os.makedirs(out_dir, exist_ok=True)
    table = {}
    for p in range(ix.ctx.num_partitions):
        recs = ix.partition_records(p)
        pos = write_sequence_file(os.path.join(out_dir, "part-%05d" % p), recs, sync)
        table[p] = [(key_of(recs, o), q) for (o, _), q in zip(iter_records(recs), pos)]
    return table


def key_grams(key):
    """TermDF bytes -> (list of writeUTF bodies, df field)."""
    k = struct.unpack_from(">i", key, 0)[0]
    p, out = 4, []
    for _ in range(k):
        ln = struct.unpack_from(">H", key, p)[0]
        out.append(key[p + 2:p + 2 + ln])
        p += 2 + ln
    return out, struct.unpack_from(">i", key, p)[0]


def mutf8_to_u16be(b):
    out, i = bytearray(), 0
    while i < len(b):
        c = b[i]
        if c < 0x80:
            u, i = c, i + 1
        elif c & 0xE0 == 0xC0:
            u, i = ((c & 0x1F) << 6) | (b[i + 1] & 0x3F), i + 2
        else:
            u, i = ((c & 0x0F) << 12) | ((b[i + 1] & 0x3F) << 6) | (b[i + 2] & 0x3F), i + 3
        out += struct.pack(">H", u)
    return bytes(out)


def termdf_sort_key(key):
    """TermDF.compareTo (TermDF.java:64-70): element-wise String.compareTo over
    UTF-16 units, then the shorter array first == tuple order of UTF-16BE bytes."""
    return tuple(mutf8_to_u16be(g) for g in key_grams(key)[0])


def build_forward_index(table, path=None):
    """BuildIntDocVectorsForwardIndex: one writeUTF(k_gram[0] \\t pos) per index
    record, in global TermDF order (one reducer).  Returns the file bytes."""
    entries = [(termdf_sort_key(key), key, p * BIG_NUMBER + pos) for p, lst in table.items() for key, pos in lst]
    entries.sort(key=lambda e: e[0])
    out = bytearray()
    for _, key, pos in entries:
        body = key_grams(key)[0][0] + b"\t" + str(pos).encode()
        if len(body) > 65535:
            raise ValueError("writeUTF: encoded string too long")  # UTFDataFormatException
        out += struct.pack(">H", len(body)) + body
    if path is not None:
        with open(path, "wb") as f:
            f.write(out)
    return bytes(out)


def read_forward_index(data):
    """IntDocVectorsForwardIndex ctor (:107-120): readUTF until EOF, split on tab,
    Hashtable.put (a later k-gram with the same first term overwrites, T11)."""
    pos, i = {}, 0
    while i + 2 <= len(data):
        ln = struct.unpack_from(">H", data, i)[0]
        if i + 2 + ln > len(data):
            break
        s = data[i + 2:i + 2 + ln]
        i += 2 + ln
        parts = s.split(b"\t")
        try:
            pos[parts[0]] = int(parts[1])
        except (IndexError, ValueError):
            break  # the ctor's catch(Exception) ends the loop
    return pos


def read_record_at(data, pos):
    """SequenceFile.Reader.seek(pos) + next(key, value): a sync block at pos is
    consumed first.  Returns (key bytes, value bytes)."""
    rl = struct.unpack_from(">i", data, pos)[0]
    if rl == SYNC_ESCAPE:
        pos += 4 + 16
        rl = struct.unpack_from(">i", data, pos)[0]
    kl = struct.unpack_from(">i", data, pos + 4)[0]
    return data[pos + 8:pos + 8 + kl], data[pos + 8 + kl:pos + 8 + rl]


def value_postings(val):
    """ArrayListWritable<PostingWritable>.readFields -> [(docno, tf), ...]."""
    n = struct.unpack_from(">i", val, 0)[0]
    if n <= 0:
        return []
    q = 6 + struct.unpack_from(">H", val, 4)[0]
    return [struct.unpack_from(">ii", val, q + 8 * j) for j in range(n)]


class ForwardIndex:
    """Term -> (k_gram, df field, postings) through the part files, as
    IntDocVectorsForwardIndex.getValue(String) does."""

    def __init__(self, index_dir, fwd_path):
        self.index_dir = index_dir
        with open(fwd_path, "rb") as f:
            self.positions = read_forward_index(f.read())
        self._files = {}

    def _file(self, no):
        if no not in self._files:
            with open(os.path.join(self.index_dir, "part-%05d" % no), "rb") as f:
                data = f.read()
            if data[:4] != b"SEQ\x06":
                raise IOError("part-%05d is not a SequenceFile v6" % no)
            self._files[no] = data
        return self._files[no]

    def get_value(self, term_mutf8):
        """None for an unknown term (getValue returns silently) or a key mismatch."""
        pos = self.positions.get(term_mutf8)
        if pos is None:
            return None
        key, val = read_record_at(self._file(pos // BIG_NUMBER), pos % BIG_NUMBER)
        grams, df = key_grams(key)
        if grams[0] != term_mutf8:
            return None  # "unable to doc vector for term": not added to keys/values
        return grams, df, value_postings(val)
