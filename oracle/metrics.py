"""Literal restatement of the reference's WER (essentials.py:576-602): full (m+1) x (n+1) distance
matrix, words lower-cased and split on whitespace.  TEST INFRASTRUCTURE ONLY (oracle/__init__.py)."""


def levenshtein(reference_words, hypothesis_words):
    m, n = len(reference_words), len(hypothesis_words)
    d = [[0] * (n + 1) for _ in range(m + 1)]
    for q in range(m + 1):
        d[q][0] = q
    for k in range(n + 1):
        d[0][k] = k
    for q in range(1, m + 1):
        for k in range(1, n + 1):
            if reference_words[q - 1] == hypothesis_words[k - 1]:
                d[q][k] = d[q - 1][k - 1]
            else:
                d[q][k] = min(d[q - 1][k - 1] + 1, d[q][k - 1] + 1, d[q - 1][k] + 1)
    return d[m][n]


def wer_batch(references, hypotheses):
    errors = words = 0
    for ref, hyp in zip(references, hypotheses):
        rw = ref.lower().split()
        errors += levenshtein(rw, hyp.lower().split())
        words += len(rw)
    return errors / words * 100 if words > 0 else 0.0
