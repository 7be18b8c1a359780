"""A user scoring plugin of the kind the reference accepts (any
``BeamScoreFunction`` subclass, `lattice_tagger/beam/score_funcs.py:7-15`):
here one that reads only the hypothesis' last word and the appended word,
declared ``edge_local`` so the build can lower it per lattice edge.

The class is made for a given base class, so the golden generator
(tests/golden/make_golden.py) runs the very same logic inside the reference
(subclassing the reference's ``BeamScoreFunction``) and the tests run it in
the build (subclassing the build's).  Test infrastructure, not product code.
"""


def make_edge_table_class(base):
    class EdgeTableScore(base):
        """``table[(wj.<field>, wk.<field>)]`` (default int 0) for appending
        ``wk`` to a hypothesis ending in ``wj``."""
        edge_local = True

        def __init__(self, table, field='tag0'):
            self.table = table
            self.field = field

        def score(self, seq, word_k):
            wj = seq.sequences[-1]
            return self.table.get((getattr(wj, self.field), getattr(word_k, self.field)), 0)

        def evaluate(self, seq):
            words = list(seq.sequences)
            total = 0
            for a, b in zip(words, words[1:]):
                total += self.table.get((getattr(a, self.field), getattr(b, self.field)), 0)
            return total

    return EdgeTableScore


def spec_of_edge(func):
    items = []
    for (a, b), v in func.table.items():
        items.append([a, b, ['i', v] if isinstance(v, int) else ['f', float(v).hex()]])
    return {'type': 'EdgeTableScore', 'field': func.field, 'items': items}


def edge_from_spec(cls, sp):
    table = {}
    for a, b, (kind, v) in sp['items']:
        table[(a, b)] = int(v) if kind == 'i' else float.fromhex(v)
    return cls(table, sp['field'])
