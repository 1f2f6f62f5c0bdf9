"""``QuasiDistr`` algebra restated — TEST INFRASTRUCTURE ONLY.

Follows ``third_party/qvm/qvm/quasi_distr.py`` line by line in behaviour:
truncation ``|v| > accuracy`` on every construction (``:3,7-10``),
``from_counts`` (``:12-20``), ``nearest_probability_distribution`` (``:28-43``),
``split`` (``:45-53``), XOR ``merge`` with overwrite on collision (``:55-60``),
``+``/``-`` (``:62-76``) and scalar ``*`` (``:78-86``). ``accuracy`` is a
per-instance setting so exact (0.0) and shipped (1e-5) behaviour can be run
side by side.
"""


class QD(dict):
    def __init__(self, data, accuracy=1e-5):
        super().__init__({k: v for k, v in data.items() if abs(v) > accuracy})
        self.acc = accuracy

    def _new(self, data):
        return QD(data, self.acc)

    @staticmethod
    def from_counts(counts, accuracy=1e-5):
        shots = sum(counts.values())
        return QD({int("".join(k.split()), 2): v / shots for k, v in counts.items()}, accuracy)

    def npd(self):
        items = sorted(self.items(), key=lambda kv: kv[1])
        n = len(items)
        beta = 0.0
        res = {}
        for k, v in items:
            if v + beta / n < 0:
                beta += v
                n -= 1
            else:
                res[k] = v + beta / n
        return res

    def split(self, bit):
        mask = 1 << bit
        a, b = {}, {}
        for k, v in self.items():
            if k & mask == 0:
                a[k] = v
            else:
                b[k & ~mask] = v
        return self._new(a), self._new(b)

    def merge(self, other):
        d = {}
        for k1, v1 in self.items():
            for k2, v2 in other.items():
                d[k1 ^ k2] = v1 * v2
        return self._new(d)

    def add(self, other):
        d = {k: self[k] + other.get(k, 0.0) for k in self}
        d.update({k: other[k] for k in other if k not in self})
        return self._new(d)

    def sub(self, other):
        d = {k: self[k] - other.get(k, 0.0) for k in self}
        d.update({k: -other[k] for k in other if k not in self})
        return self._new(d)

    def scale(self, x):
        return self._new({k: v * x for k, v in self.items()})
