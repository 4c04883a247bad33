"""Pure-Python restatement of NuPIC 1.0.x RandomDistributedScalarEncoder.

TEST INFRASTRUCTURE ONLY: a second, independent restatement of the encoder of
the reference's model.yaml parameter set (ML/HTM/params/model.yaml:15-21,
``type: RandomDistributedScalarEncoder, resolution: 0.88, seed: 1``), kept in
the shape of NuPIC's nupic/encoders/random_distributed_scalar.py (a dict
bucket map grown by the recursive _createBucket, _newRepresentation's redraw
loop, _newRepresentationOK's running overlap) with a pure-Python
nupic::Random, so that tests can hold the C oracle's
loop form (oracle/htm_oracle.c rdse_*) against it.  NuPIC itself is absent
(SURVEY.md §8(c)): parity w.r.t. NuPIC is unpinned.
"""
import math

INITIAL_BUCKETS = 1000


class NupicRandom:
    """nupic::Random (BSD random() TYPE_3, 31 words, separation 3)."""

    def __init__(self, seed):
        x = seed % 2147483646 + 1
        s = [x]
        for _ in range(1, 31):
            hi, lo = divmod(x, 127773)
            x = 16807 * lo - 2836 * hi
            if x < 0:
                x += 2147483647
            s.append(x)
        self.s, self.f, self.r = s, 3, 0
        for _ in range(310):
            self._raw()

    def _raw(self):
        s = self.s
        s[self.f] = (s[self.f] + s[self.r]) & 0xFFFFFFFF
        i = (s[self.f] >> 1) & 0x7FFFFFFF
        self.f += 1
        if self.f >= 31:
            self.f = 0
            self.r += 1
        else:
            self.r += 1
            if self.r >= 31:
                self.r = 0
        return i

    def getUInt32(self, n):
        smax = 0xFFFFFFFF - (0xFFFFFFFF % n)
        while True:
            v = self._raw()
            if v <= smax:
                return v % n

    def shuffle(self, arr):
        """Random.hpp shuffle: swap(first[0], first[getUInt32(n)]), n decreasing."""
        n = len(arr)
        for i in range(len(arr)):
            j = self.getUInt32(n)
            arr[i], arr[i + j] = arr[i + j], arr[i]
            n -= 1


def py2_round(v):
    """Python 2's round(): halves away from zero."""
    t = math.trunc(v)
    fr = v - t
    if fr >= 0.5:
        return t + 1
    if fr <= -0.5:
        return t - 1
    return t


class RDSE:
    def __init__(self, resolution, w=21, n=400, offset=None, seed=42):
        if w <= 0 or w % 2 == 0:
            raise ValueError("w must be an odd positive integer")
        if n <= 6 * w:
            raise ValueError("n must be an int strictly greater than 6*w")
        self.w, self.n, self.resolution = w, n, float(resolution)
        self._maxOverlap = 2
        self.random = NupicRandom(seed)
        self.numTries = 0
        self._maxBuckets = INITIAL_BUCKETS
        self.minIndex = self._maxBuckets // 2
        self.maxIndex = self._maxBuckets // 2
        self._offset = offset
        self.bucketMap = {}
        r = list(range(self.n))
        self.random.shuffle(r)
        self.bucketMap[self.minIndex] = r[0:self.w]

    def getBucketIndices(self, x):
        if x is None or (isinstance(x, float) and math.isnan(x)):
            return [None]
        if self._offset is None:
            self._offset = x
        idx = self._maxBuckets // 2 + int(py2_round((x - self._offset) / self.resolution))
        return [min(max(idx, 0), self._maxBuckets - 1)]

    def mapBucketIndexToNonZeroBits(self, index):
        index = min(max(index, 0), self._maxBuckets - 1)
        if index not in self.bucketMap:
            self._createBucket(index)
        return self.bucketMap[index]

    def encode(self, x):
        out = [0] * self.n
        b = self.getBucketIndices(x)[0]
        if b is not None:
            for bit in self.mapBucketIndexToNonZeroBits(b):
                out[bit] = 1
        return out, b

    def _createBucket(self, index):
        if index < self.minIndex:
            if index == self.minIndex - 1:
                self.bucketMap[index] = self._newRepresentation(self.minIndex, index)
                self.minIndex = index
            else:
                self._createBucket(index + 1)
                self._createBucket(index)
        else:
            if index == self.maxIndex + 1:
                self.bucketMap[index] = self._newRepresentation(self.maxIndex, index)
                self.maxIndex = index
            else:
                self._createBucket(index - 1)
                self._createBucket(index)

    def _newRepresentation(self, index, newIndex):
        newRepresentation = list(self.bucketMap[index])
        ri = newIndex % self.w
        newBit = self.random.getUInt32(self.n)
        newRepresentation[ri] = newBit
        while newBit in self.bucketMap[index] or not self._newRepresentationOK(newRepresentation, newIndex):
            self.numTries += 1
            newBit = self.random.getUInt32(self.n)
            newRepresentation[ri] = newBit
        return newRepresentation

    def _newRepresentationOK(self, newRep, newIndex):
        if len(newRep) != self.w:
            return False
        newRepBinary = [False] * self.n
        for b in newRep:
            newRepBinary[b] = True
        midIdx = self._maxBuckets // 2
        runningOverlap = sum(1 for e in self.bucketMap[self.minIndex] if e in newRep)
        if not self._overlapOK(self.minIndex, newIndex, runningOverlap):
            return False
        for i in range(self.minIndex + 1, midIdx + 1):
            newBit = (i - 1) % self.w
            if newRepBinary[self.bucketMap[i - 1][newBit]]:
                runningOverlap -= 1
            if newRepBinary[self.bucketMap[i][newBit]]:
                runningOverlap += 1
            if not self._overlapOK(i, newIndex, runningOverlap):
                return False
        for i in range(midIdx + 1, self.maxIndex + 1):
            newBit = i % self.w
            if newRepBinary[self.bucketMap[i - 1][newBit]]:
                runningOverlap -= 1
            if newRepBinary[self.bucketMap[i][newBit]]:
                runningOverlap += 1
            if not self._overlapOK(i, newIndex, runningOverlap):
                return False
        return True

    def _overlapOK(self, i, j, overlap):
        if abs(i - j) < self.w:
            return overlap == self.w - abs(i - j)
        return overlap <= self._maxOverlap
