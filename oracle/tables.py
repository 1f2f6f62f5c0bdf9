"""Virtual-gate instantiation tables and knit rules — TEST INFRASTRUCTURE ONLY.

Restated from ``third_party/qvm/qvm/virtual_gates.py`` (line numbers per
entry). An instantiation is ``(side0_ops, side1_ops)``; an op is
``(name, params)`` or ``"M"`` (measure into the gate's config clbit). Each
rule takes ``results`` (list of :class:`oracle.quasi.QD`) and the config
``clbit`` and evaluates exactly the reference's expression, in its
association order.
"""
from math import cos, pi, sin

RZZ_ACCURACY = 0.00001  # virtual_gates.py:223


def _cz_table():  # virtual_gates.py:154-177
    return [
        ([("sdg", ())], [("sdg", ())]),
        ([("s", ())], [("s", ())]),
        (["M"], []),
        (["M"], [("z", ())]),
        ([], ["M"]),
        ([("z", ())], ["M"]),
    ]


def table(kind, params=()):
    if kind == "cz":
        return _cz_table()
    if kind == "cx":  # virtual_gates.py:197-206: h on qubit 1 before and after
        return [(a, [("h", ())] + b + [("h", ())]) for a, b in _cz_table()]
    if kind == "cy":  # virtual_gates.py:209-220: rz(-pi/2) . CX-inst . rz(pi/2) on qubit 1
        return [(a, [("rz", (-pi / 2,))] + b + [("rz", (pi / 2,))]) for a, b in table("cx")]
    if kind == "rzz":  # virtual_gates.py:230-260
        mt = -params[0]
        if abs(cos(mt / 2)) < RZZ_ACCURACY:
            return [([("z", ())], [("z", ())])]
        if abs(sin(mt / 2)) < RZZ_ACCURACY:
            return [([], [])]
        return [
            ([], []),
            ([("z", ())], [("z", ())]),
            ([("rz", (-pi / 2,))], ["M"]),
            (["M"], [("rz", (-pi / 2,))]),
            ([("rz", (pi / 2,))], ["M"]),
            (["M"], [("rz", (pi / 2,))]),
        ]
    if kind == "cp":  # virtual_gates.py:294-310; params are the already-rewritten (-lambda/2)
        lam = params[0]
        return [([("rz", (lam / 2,))] + a, b + [("rz", (lam / 2,))]) for a, b in table("rzz", params)]
    if kind == "move":  # virtual_gates.py:62-103
        return [
            ([], []),
            ([], [("x", ())]),
            ([("h", ()), "M"], [("h", ())]),
            ([("h", ()), "M"], [("x", ()), ("h", ())]),
            ([("sdg", ()), ("h", ()), "M"], [("h", ()), ("s", ())]),
            ([("sdg", ()), ("h", ()), "M"], [("x", ()), ("h", ()), ("s", ())]),
            (["M"], []),
            (["M"], [("x", ())]),
        ]
    raise ValueError(kind)


def _signed_sum(results, clbit, signs):
    acc = None
    for s, r in zip(signs, results):
        a, b = r.split(clbit)
        term = a.sub(b)
        if acc is None:
            acc = term  # first term enters unchanged (+)
        else:
            acc = acc.add(term) if s > 0 else acc.sub(term)
    return acc.scale(0.5)


def knit(kind, params, results, clbit):
    if kind in ("cz", "cx", "cy"):  # virtual_gates.py:179-194
        return _signed_sum(results, clbit, (1, 1, 1, -1, 1, -1))
    if kind == "move":  # virtual_gates.py:105-124
        return _signed_sum(results, clbit, (1, 1, 1, -1, 1, -1, 1, -1))
    if kind in ("rzz", "cp"):  # virtual_gates.py:262-286
        mt = -params[0]
        c, s = cos(mt / 2), sin(mt / 2)
        if abs(c) < RZZ_ACCURACY:
            return results[0].split(clbit)[0].scale(s ** 2)
        if abs(s) < RZZ_ACCURACY:
            return results[0].split(clbit)[0].scale(c ** 2)
        r0 = results[0].split(clbit)[0]
        r1 = results[1].split(clbit)[0]
        r230, r231 = results[2].add(results[3]).split(clbit)
        r450, r451 = results[4].add(results[5]).split(clbit)
        mix = r230.sub(r231).sub(r450).add(r451)
        return r0.scale(c ** 2).add(r1.scale(s ** 2)).add(mix.scale(c).scale(s))
    raise ValueError(kind)


def coefficients(kind, params):
    """Per-instantiation coefficient with config outcomes folded as (-1)^m (dense form)."""
    if kind in ("cz", "cx", "cy"):
        return [0.5 * x for x in (1, 1, 1, -1, 1, -1)]
    if kind == "move":
        return [0.5 * x for x in (1, 1, 1, -1, 1, -1, 1, -1)]
    mt = -params[0]
    c, s = cos(mt / 2), sin(mt / 2)
    if abs(c) < RZZ_ACCURACY:
        return [s * s]
    if abs(s) < RZZ_ACCURACY:
        return [c * c]
    return [c * c, s * s, c * s, c * s, -c * s, -c * s]
