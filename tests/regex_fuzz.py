"""Random valid patterns/contents for cross-checking the product's engine and
lowering (C-ABI fr_plain_match) against oracle/regex_oracle.py."""
import random

LETTERS = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ"
SYMS = "&;:,`~-_!@#%'\""


def rand_ext_class(rng):
    """A bracket class of the grammar extension (FR_GRAMMAR_EXT)."""
    items = []
    for _ in range(rng.randint(1, 3)):
        k = rng.random()
        if k < 0.4:
            a, b = sorted(rng.sample("0123456789", 2))
        elif k < 0.7:
            a, b = sorted(rng.sample("abcdexyz", 2))
        else:
            a = b = rng.choice("0159aAz_\\-")
        items.append(a if a == b else f"{a}-{b}")
    body = "".join("\\-" if it == "-" else ("\\\\" if it == "\\" else it) for it in items)
    return "[" + ("^" if rng.random() < 0.3 else "") + body + "]"


def rand_atom(rng, depth, ext=False):
    if ext and rng.random() < 0.3:
        return rng.choice("0123") if rng.random() < 0.3 else rand_ext_class(rng)
    r = rng.random()
    if r < 0.45:
        return rng.choice("abcdeABC")
    if r < 0.52:
        return "."
    if r < 0.58:
        return "\\" + rng.choice("0123456789.*^$")
    if r < 0.62:
        return rng.choice(SYMS)
    if r < 0.80:
        k = rng.random()
        if k < 0.35:
            a, b = sorted(rng.sample("abcdefgh", 2))
            return f"[{a}-{b}]"
        if k < 0.7:
            return "[" + "".join(rng.sample("abcdeXYZ", rng.randint(1, 3))) + "]"
        if k < 0.85:
            a, b = sorted(rng.sample("abcdefgh", 2))
            return f"[^{a}-{b}]"
        return "[^" + "".join(rng.sample("abcxyz", rng.randint(1, 3))) + "]"
    if depth < 2:
        return "(" + rand_regex(rng, depth + 1, ext) + ")"
    return rng.choice("abc")


def rand_factor(rng, depth, ext=False):
    a = rand_atom(rng, depth, ext)
    r = rng.random()
    if r < 0.6:
        return a
    if r < 0.7:
        return a + "?"
    if r < 0.78:
        return a + "*"
    if r < 0.86:
        return a + "+"
    if r < 0.92:
        return a + "{%d}" % rng.randint(0, 3)
    lo = rng.choice(["", str(rng.randint(0, 2))])
    hi = rng.choice(["", str(rng.randint(1, 3))])
    return a + "{%s,%s}" % (lo, hi)


def rand_term(rng, depth, ext=False):
    return "".join(rand_factor(rng, depth, ext) for _ in range(rng.randint(1, 3)))


def rand_regex(rng, depth=0, ext=False):
    t = rand_term(rng, depth, ext)
    if rng.random() < 0.25:
        t += "|" + rand_term(rng, depth, ext)
    return t


def rand_pattern(rng, ext=False):
    p = "/" + ("^" if rng.random() < 0.25 else "") + rand_regex(rng, 0, ext) + ("$" if rng.random() < 0.25 else "") + "/"
    if rng.random() < 0.2:
        p += "i"
    return p


def rand_content(rng, n):
    return "".join(rng.choice("abcdeABCxyz0.* ") for _ in range(n))
