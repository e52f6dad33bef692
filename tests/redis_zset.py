"""An independent model of the Redis sorted set behind NFIRankRedisModule (test infrastructure):
NFCRankRedisModule::GetRange (NFCRankRedisModule.cpp:109) is ZREVRANGE key 0 k-1 WITHSCORES over
members NFGUID::ToString() ("head-data", NFGUID.h:93).  Redis keeps a skiplist ordered by (score,
member) ascending, members compared as bytes (memcmp, shorter prefix first); ZREVRANGE walks it
from the tail.  This restates that with an explicit comparator, independently of shard.zrevrange_order."""
import functools


def _cmp(a, b):
    """zslInsert / zslGetRank order: score, then sdscmp of the member bytes"""
    if a[0] != b[0]:
        return -1 if a[0] < b[0] else 1
    if a[1] == b[1]:
        return 0
    return -1 if a[1] < b[1] else 1   # bytes compare like memcmp with the length as the tiebreak


class ZSet:
    def __init__(self):
        self._k = {}      # member bytes -> score (ZADD updates a member's score)
        self._sorted = None

    def zadd(self, member, score):
        self._k[member.encode()] = float(score) + 0.0   # (-0.0 and 0.0 are one score in a skiplist)
        self._sorted = None

    def zrevrange(self, start, stop):
        if self._sorted is None:   # the skiplist's order, ascending
            self._sorted = sorted(((s, m) for m, s in self._k.items()), key=functools.cmp_to_key(_cmp))
        rev = self._sorted[::-1]
        stop = len(rev) - 1 if stop < 0 else stop
        return [(m.decode(), s) for s, m in rev[start:stop + 1]]


def zrevrange_top(gh, gd, score, k):
    """indices of the top k entries (members "head-data") in ZREVRANGE order"""
    z = ZSet()
    idx = {}
    for i in range(len(score)):
        m = f"{int(gh[i])}-{int(gd[i])}"
        idx[m] = i
        z.zadd(m, score[i])
    return [idx[m] for m, _ in z.zrevrange(0, k - 1)]
