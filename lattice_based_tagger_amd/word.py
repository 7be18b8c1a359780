"""Lattice node type.

`Word` has the field layout of the reference lattice node
(`lattice_tagger/dictionary/dictionary.py:169-199`):
``word morph0 morph1 tag0 tag1 len b e is_l``.  The decoder never relies on
the concrete class: any object with these attributes (in particular the
reference's own ``Word``) is accepted as a lattice node.
"""

from collections import namedtuple

from .tagset import BOS, EOS, Unk

_WordBase = namedtuple('Word', 'word morph0 morph1 tag0 tag1 len b e is_l')


class Word(_WordBase):
    __slots__ = ()

    def __str__(self):
        tail = ', L' if self.is_l else ''
        if self.morph1:
            return 'Word(%s, %s/%s + %s/%s, len=%d, b=%d, e=%d%s)' % (
                self.word, self.morph0, self.tag0, self.morph1, self.tag1,
                self.len, self.b, self.e, tail)
        return 'Word(%s, %s/%s, len=%d, b=%d, e=%d%s)' % (
            self.word, self.morph0, self.tag0, self.len, self.b, self.e, tail)

    __repr__ = __str__


def bos_word():
    """Sentence-start sentinel (`beam/beam.py:21`)."""
    return Word(BOS, BOS, None, BOS, None, 0, 0, 0, False)


def eos_word(n):
    """Sentence-end sentinel for an n-character sentence (`beam/beam.py:22`)."""
    return Word(EOS, EOS, None, EOS, None, 0, n, n, False)


def unknown_word(chars, b, e):
    """The node the decoder synthesises for a span with no dictionary
    candidate (`beam/beam.py:36-38`)."""
    sub = chars[b:e]
    return Word(sub, sub, None, Unk, None, e - b, b, e, False)
