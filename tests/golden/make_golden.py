"""Generates tests/golden/parser_vectors.json and engine_vectors.json.

The (pattern -> AST) cases are transcribed from the reference's own parser
tests, src/regex/parser.rs:358-678 (49 #[test_case]s), into the canonical AST
string form of oracle/regex_oracle.py.  The (content, pattern, expected) cases
are src/regex/engine.rs:256-280; ct_ops/cache_hits are SURVEY.md Appendix B
(hand-derived from the reference source, not from a run).  Pure data: no
reference source is copied.
"""
import json, os

C = lambda ch: f"Char({ord(ch)})"
def seq(*xs): return "Seq(" + ",".join(xs) + ")"
abc = seq(C("a"), C("b"), C("c"))

parser = [
    ("/h/", C("h"), "char"),
    ("/&/", C("&"), "ampersand"), ("/;/", C(";"), "semicolon"), ("/:/", C(":"), "colon"),
    ("/,/", C(","), "comma"), ("/`/", C("`"), "backtick"), ("/~/", C("~"), "tilde"),
    ("/-/", C("-"), "minus"), ("/_/", C("_"), "underscore"), ("/%/", C("%"), "percentage"),
    ("/#/", C("#"), "hashtag"), ("/@/", C("@"), "at"), ("/!/", C("!"), "exclamation"),
    ("/'/", C("'"), "single quote"), ('/"/', C('"'), "double quote"),
    ("/\\h/", C("h"), "anything can be escaped"),
    ("/./", "Any", "any"),
    ("/abc/", abc, "abc"),
    ("/^abc/", seq("SOF", abc), "<sof>abc"),
    ("/abc$/", seq(abc, "EOF"), "abc<eof>"),
    ("/^abc$/", seq("SOF", abc, "EOF"), "<sof>abc<eof>"),
    ("/^ab?c$/", seq("SOF", seq(C("a"), f"Optional({C('b')})", C("c")), "EOF"), "question"),
    ("/^ab*c$/", seq("SOF", seq(C("a"), f"Repeated({C('b')},_,_)", C("c")), "EOF"), "star"),
    ("/^ab+c$/", seq("SOF", seq(C("a"), f"Repeated({C('b')},1,_)", C("c")), "EOF"), "plus"),
    ("/^ab{2}c$/", seq("SOF", seq(C("a"), f"Repeated({C('b')},2,2)", C("c")), "EOF"), "twice"),
    ("/^ab{3,}c$/", seq("SOF", seq(C("a"), f"Repeated({C('b')},3,_)", C("c")), "EOF"), "atleast 3"),
    ("/^ab{2,4}c$/", seq("SOF", seq(C("a"), f"Repeated({C('b')},2,4)", C("c")), "EOF"), "between 2 and 4"),
    ("/^.$/", seq("SOF", "Any", "EOF"), "<sof><any><eof>"),
    ("/^[abc]$/", seq("SOF", "Range(97,98,99)", "EOF"), "a or b or c"),
    ("/^[a-d]$/", seq("SOF", "Between(97,100)", "EOF"), "between a and d"),
    ("/^[^abc]$/", seq("SOF", "Not(Range(97,98,99))", "EOF"), "not a or b or c"),
    ("/^[^a-d]$/", seq("SOF", "Not(Between(97,100))", "EOF"), "not between a and d"),
    ("/^abc$/i", seq("SOF", seq("Range(97,65)", "Range(98,66)", "Range(99,67)"), "EOF"), "case insensitive"),
    ("/^/", seq("SOF", "Seq()"), "sof"),
    ("/$/", seq("Seq()", "EOF"), "eof"),
    ("/a*/", f"Repeated({C('a')},_,_)", "repeat unbounded"),
    ("/a+/", f"Repeated({C('a')},1,_)", "repeat at least 1"),
    ("/a{104,}/", f"Repeated({C('a')},104,_)", "repeat at least x"),
    ("/a{,15}/", f"Repeated({C('a')},_,15)", "repeat at most x"),
    ("/a{12,15}/", f"Repeated({C('a')},12,15)", "repeat between"),
    ("/(a|b)*/", f"Repeated(Either({C('a')},{C('b')}),_,_)", "repeat complex unbounded"),
    ("/(a|b){3,7}/", f"Repeated(Either({C('a')},{C('b')}),3,7)", "repeat complex bounded"),
    ("/^ab|cd/", seq("SOF", f"Either({seq(C('a'), C('b'))},{seq(C('c'), C('d'))})"), "SOF encapsulates full RHS"),
    ("/ab|cd$/", seq(f"Either({seq(C('a'), C('b'))},{seq(C('c'), C('d'))})", "EOF"), "EOF encapsulates full RHS"),
    ("/^ab|cd$/", seq("SOF", f"Either({seq(C('a'), C('b'))},{seq(C('c'), C('d'))})", "EOF"), "SOF + EOF"),
    ("/\\^/", C("^"), "escaping sof symbol"),
    ("/\\./", C("."), "escaping period"),
    ("/\\*/", C("*"), "escaping star"),
    ("/^ca\\^b$/", seq("SOF", seq(C("c"), C("a"), C("^"), C("b")), "EOF"), "escaping, more realistic"),
]
assert len(parser) == 49, len(parser)

# (content, pattern, expected) : engine.rs:256-280 ; (ct_ops, cache_hits): SURVEY App. B
engine = [
    ("ab", "/ab/", 1, 3, 0), ("b", "/ab/", 0, 0, 0), ("ab", "/a?b/", 1, 6, 1), ("b", "/a?b/", 1, 1, 0),
    ("ab", "/^ab|cd$/", 1, 7, 0), (" ab", "/^ab|cd$/", 0, 0, 0), (" cd", "/^ab|cd$/", 0, 0, 0),
    ("cd", "/^ab|cd$/", 1, 7, 0), ("abcd", "/^ab|cd$/", 0, 0, 0), ("abcd", "/ab|cd$/", 1, 7, 0),
    ("abc", "/abc/", 1, 5, 0), ("123abc", "/abc/", 1, 23, 0), ("123abc456", "/abc/", 1, 41, 0),
    ("123abdc456", "/abc/", 0, 47, 0), ("abc456", "/abc/", 1, 23, 0), ("bc", "/a*bc/", 1, 3, 0),
    ("cdaabc", "/a*bc/", 1, 59, 40), ("cdbc", "/a+bc/", 0, 15, 4), ("bc", "/a+bc/", 0, 0, 0),
    ("Ab", "/ab/i", 1, 7, 0), ("Ab", "/ab/", 0, 3, 0), ("cD", "/ab|cd/i", 1, 15, 0),
    ("cD", "/cD/", 1, 3, 0), ("de", "/^ab|cd|de$/", 1, 11, 0), (" de", "/^ab|cd|de$/", 0, 0, 0),
]
assert len(engine) == 25

here = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(here, "parser_vectors.json"), "w") as f:
    json.dump([{"pattern": p, "ast": a, "name": n} for (p, a, n) in parser], f, indent=1)
with open(os.path.join(here, "engine_vectors.json"), "w") as f:
    json.dump([{"content": c, "pattern": p, "expected": e, "ct_ops": o, "cache_hits": h,
                "source": "src/regex/engine.rs:256-280; counts SURVEY App. B"} for (c, p, e, o, h) in engine], f, indent=1)
print("ok")
