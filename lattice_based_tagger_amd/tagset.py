"""Tag vocabulary of the lattice tagger.

Same string constants as the reference tag set
(`lattice_tagger/tagset.py:1-15`): ten part-of-speech tags, the two sentinel
tags and the tag the decoder gives to synthesised unknown words.
"""

Noun = 'Noun'
Pronoun = 'Pronoun'
Number = 'Number'
Josa = 'Josa'
Adjective = 'Adjective'
Verb = 'Verb'
Eomi = 'Eomi'
Adverb = 'Adverb'
Determiner = 'Determiner'
Exclamation = 'Exclamation'

BOS = 'BOS'
EOS = 'EOS'

Unk = 'Unknown'

# Tags that make the trigram "contextual" feature (class 8) fire
# (`features/feature.py:92`).
CONTEXTUAL_TAGS = frozenset({Noun, Adverb, Adjective, Verb})

POS_TAGS = (Noun, Pronoun, Number, Josa, Adjective, Verb, Eomi, Adverb,
            Determiner, Exclamation)

__all__ = ['Noun', 'Pronoun', 'Number', 'Josa', 'Adjective', 'Verb', 'Eomi',
           'Adverb', 'Determiner', 'Exclamation', 'BOS', 'EOS', 'Unk',
           'CONTEXTUAL_TAGS', 'POS_TAGS']
