"""A subset Go type checker for the drop-in's Go files (test infrastructure: there is no Go
toolchain in this image, so go vet / go build never run on them).

It parses the Go the drop-in is written in (gofmt-formatted package code: declarations,
statements, expressions, function literals, composite literals) and type-checks what a compiler
would reject in it:
  * every identifier resolves (locals with block scoping, package scope, imports, universe);
  * every selector x.f names a field or method of x's type, including fields and methods promoted
    through embedded structs (batchManager embeds *manager);
  * calls pass as many arguments as the function takes, and each argument is assignable to its
    parameter; for cgo calls the parameter types come from the C prototypes in include/*.h under
    cgo's mapping (uint8_t* -> *C.uint8_t, const T* const* -> **C.T, void* -> unsafe.Pointer,
    integer macros -> untyped constants), so an int passed where C.int is expected is caught;
  * assignments, := declarations (including comma-ok forms), returns and composite-literal fields
    agree in count and are assignable; binary operators see identical operand types;
  * `var _ I = &T{}` assertions hold: T's method set (with promotion and pointer receivers)
    has every method of I with an identical signature;
  * no local variable is declared and never read, and no import goes unused (Go rejects both);
  * every function with results ends in a terminating statement (Go's "missing return"), and if
    conditions are boolean.

Types of the reference's own packages (internal/fec, internal/wire, internal/protocol, patched as
go/patches/*.diff patch them) come from their declarations, with type aliases resolved; packages
that are not loaded (the standard library beyond a small table, cgo's runtime helpers) and type
parameters of generic code give an unknown type, which is never reported: the checker errs
towards silence, and the tests pin its reach (how many selectors, calls and cgo arguments it
typed), its teeth (seeded errors it must report) and its silence (the reference's own packages,
Go that compiles, check clean)."""
import os
import re

# ----------------------------------------------------------------------------- lexing

KEYWORDS = {"break", "case", "chan", "const", "continue", "default", "defer", "else", "fallthrough",
            "for", "func", "go", "goto", "if", "import", "interface", "map", "package", "range",
            "return", "select", "struct", "switch", "type", "var"}
SEMI_AFTER_KW = {"break", "continue", "fallthrough", "return"}

TOKEN_RE = re.compile(r"""
    (?P<ws>[ \t\r]+)
  | (?P<nl>\n)
  | (?P<id>[A-Za-z_][A-Za-z_0-9]*)
  | (?P<num>0[xX][0-9a-fA-F_]+|0[bB][01_]+|0[oO][0-7_]+|(?:[0-9][0-9_]*(?:\.[0-9_]*)?|\.[0-9][0-9_]*)(?:[eE][+-]?[0-9]+)?)
  | (?P<str>"(?:[^"\\\n]|\\.)*"|`[^`]*`)
  | (?P<rune>'(?:[^'\\\n]|\\.[^'\n]*)')
  | (?P<op>\.\.\.|<<=|>>=|&\^=|&&|\|\||<-|\+\+|--|==|!=|<=|>=|:=|<<|>>|&\^|[-+*/%&|^]=|[-+*/%&|^<>=!.,;:(){}\[\]~])
""", re.X)


def strip_comments(src):
    """Go source with comments replaced by spaces (newlines kept, so line numbers hold)."""
    out, i, n = [], 0, len(src)
    while i < n:
        c = src[i]
        if src.startswith("//", i):
            j = src.find("\n", i)
            j = n if j < 0 else j
            out.append(" " * (j - i))
            i = j
        elif src.startswith("/*", i):
            j = src.find("*/", i + 2)
            j = n if j < 0 else j + 2
            out.append("".join(ch if ch == "\n" else " " for ch in src[i:j]))
            i = j
        elif c in "\"`'":
            j = i + 1
            while j < n and src[j] != c:
                if src[j] == "\\" and c != "`":
                    j += 1
                j += 1
            out.append(src[i:j + 1])
            i = j + 1
        else:
            out.append(c)
            i += 1
    return "".join(out)


class Tok:
    __slots__ = ("kind", "text", "line")

    def __init__(self, kind, text, line):
        self.kind, self.text, self.line = kind, text, line

    def __repr__(self):
        return "%s@%d" % (self.text, self.line)


def tokenize(src):
    """Tokens with Go's automatic semicolons (a ';' token at a line end after an identifier,
    literal, break/continue/fallthrough/return, ++, --, ), ] or })."""
    src = strip_comments(src)
    toks, line, pos = [], 1, 0
    while pos < len(src):
        m = TOKEN_RE.match(src, pos)
        if not m:
            raise SyntaxError("line %d: cannot lex %r" % (line, src[pos:pos + 20]))
        kind = m.lastgroup
        text = m.group(kind)
        pos = m.end()
        if kind == "ws":
            continue
        if kind == "nl":
            if toks and _semi_after(toks[-1]):
                toks.append(Tok("op", ";", line))
            line += 1
            continue
        if kind == "str":
            line += text.count("\n")
        toks.append(Tok(kind, text, line))
    if toks and _semi_after(toks[-1]):
        toks.append(Tok("op", ";", line))
    toks.append(Tok("eof", "", line))
    return toks


def _semi_after(t):
    if t.kind == "id":
        return t.text not in KEYWORDS or t.text in SEMI_AFTER_KW
    if t.kind in ("num", "str", "rune"):
        return True
    return t.text in ("++", "--", ")", "]", "}")


# ----------------------------------------------------------------------------- types

UNKNOWN = ("?",)
INT_NAMES = {"int", "int8", "int16", "int32", "int64", "uint", "uint8", "uint16", "uint32", "uint64",
             "uintptr", "byte", "rune"}
FLOAT_NAMES = {"float32", "float64"}
BUILTIN_TYPES = INT_NAMES | FLOAT_NAMES | {"bool", "string", "error", "any", "complex64", "complex128"}
C_NUMERIC = {"int", "uint", "long", "ulong", "longlong", "ulonglong", "short", "ushort", "char", "schar",
             "uchar", "size_t", "ssize_t", "float", "double", "uintptr_t", "intptr_t"} | {
    "%sint%d_t" % (u, b) for u in ("", "u") for b in (8, 16, 32, 64)}
BUILTIN_FUNCS = {"len", "cap", "append", "make", "new", "copy", "delete", "clear", "panic", "print",
                 "println", "min", "max", "close", "recover", "complex", "real", "imag"}


def named(pkg, name):
    if pkg == "" and name == "byte":
        name = "uint8"
    if pkg == "" and name == "rune":
        name = "int32"
    return ("named", pkg, name)


def untyped(kind):
    return ("untyped", kind)


def fmt_type(t):
    k = t[0]
    if k == "named":
        return ("%s.%s" % (t[1], t[2])) if t[1] else t[2]
    if k == "ptr":
        return "*" + fmt_type(t[1])
    if k == "slice":
        return "[]" + fmt_type(t[1])
    if k == "array":
        return "[N]" + fmt_type(t[1])
    if k == "map":
        return "map[%s]%s" % (fmt_type(t[1]), fmt_type(t[2]))
    if k == "func":
        return "func(%s) (%s)" % (", ".join(map(fmt_type, t[1])), ", ".join(map(fmt_type, t[2])))
    if k == "untyped":
        return "untyped " + t[1]
    if k == "tuple":
        return "(%s)" % ", ".join(map(fmt_type, t[1]))
    if k == "typeval":
        return "type " + fmt_type(t[1])
    return k


class GoError(Exception):
    pass


class FileCtx:
    def __init__(self, path, pkg, imports):
        self.path, self.pkg, self.imports = path, pkg, imports


class Universe:
    """Declarations of the loaded packages, C prototypes and a small standard-library table."""

    def __init__(self):
        self.types = {}      # (pkg, name) -> underlying type ('struct', fields) / ('iface', ...) / type
        self.methods = {}    # (pkg, name) -> {method: (functype, ptr_receiver)}
        self.funcs = {}      # (pkg, name) -> functype
        self.values = {}     # (pkg, name) -> type, or ('lazy', tokens, ctx)
        self.loaded = set()  # packages whose declarations are loaded
        self.cfuncs = {}     # C function -> functype
        self.cmacros = set()
        self.ctypes = set()  # C typedef names (opaque structs)
        self.bodies = []     # (ctx, FuncDecl) of the files to check
        self.import_errors = []
        self.aliases = {}    # (pkg, name) -> the aliased type (type A = B)
        self.decl_sites = {}  # (pkg, name) -> [file:line]
        self.final = False

    # -- C headers
    def load_c_header(self, text):
        text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
        text = re.sub(r"//[^\n]*", " ", text)
        for m in re.finditer(r"#define\s+([A-Z_][A-Z0-9_]*)\s+\(?-?\d+\)?", text):
            self.cmacros.add(m.group(1))
        for m in re.finditer(r"typedef\s+struct\s+\w+\s+(\w+)\s*;", text):
            self.ctypes.add(m.group(1))
        body = re.sub(r"#[^\n]*", " ", text)
        for m in re.finditer(r"([A-Za-z_][\w \t\*]*?)\b(fec_\w+)\s*\(([^()]*)\)\s*;", body):
            ret, name, params = m.group(1), m.group(2), m.group(3).strip()
            ps = [] if params in ("", "void") else [self._c_param(p) for p in params.split(",")]
            r = self._c_type(ret)
            self.cfuncs[name] = ("func", tuple(ps), () if r is None else (r,), False)

    def _c_param(self, p):
        p = p.strip()
        m = re.match(r"^(.*?)([A-Za-z_]\w*)\s*(\[\s*\])?$", p)
        if m and m.group(1).strip() and m.group(1).strip() not in ("const", "unsigned", "struct"):
            base = m.group(1) + ("*" if m.group(3) else "")
        else:
            base = p
        t = self._c_type(base)
        return UNKNOWN if t is None else t

    def _c_type(self, text):
        stars = text.count("*")
        words = [w for w in re.findall(r"[A-Za-z_]\w*", text) if w not in ("const", "extern", "static", "inline", "struct")]
        if not words:
            return UNKNOWN
        if words[:2] == ["unsigned", "char"]:
            base = "uchar"
        elif words[:2] == ["unsigned", "int"] or words == ["unsigned"]:
            base = "uint"
        elif words[:2] == ["long", "long"]:
            base = "longlong"
        else:
            base = words[-1]
        if base == "void":
            if stars == 0:
                return None
            t, stars = named("unsafe", "Pointer"), stars - 1
        else:
            t = named("C", base)
        for _ in range(stars):
            t = ("ptr", t)
        return t

    # -- Go files
    def load_go(self, path, src, check=False):
        """check: False (declarations only), True (every function body), or a set of line
        numbers (the bodies of the functions spanning one of them)."""
        toks = tokenize(src)
        p = DeclParser(self, path, toks, check)
        p.parse_file()
        self.loaded.add(p.ctx.pkg)
        if check:   # an import no code of the file names is a compile error
            named_ = {toks[i].text for i in range(len(toks) - 1) if toks[i].kind == "id" and toks[i + 1].text == "."}
            for alias in p.ctx.imports:
                if alias not in ("_", ".") and alias not in named_:
                    self.import_errors.append("%s: imported and not used: %s" % (os.path.basename(path), alias))
        return p.ctx

    def underlying(self, t, depth=0):
        while t[0] == "named" and depth < 20:
            if t[1] == "" and t[2] in BUILTIN_TYPES:
                if t[2] == "error":
                    return ("iface", {"Error": (("func", (), (named("", "string"),), False), False)}, ())
                if t[2] == "any":
                    return ("iface", {}, ())
                return t
            if t[1] == "C":
                return t
            u = self.types.get((t[1], t[2]))
            if u is None:
                return UNKNOWN
            t = u
            depth += 1
        return t

    def is_loaded(self, pkg):
        return pkg == "" or pkg in self.loaded

    def canon(self, t, depth=0):
        """t with every alias replaced by the type it names (type A = B: A and B are identical)."""
        if depth > 20 or not isinstance(t, tuple) or not t:
            return t
        k = t[0]
        if k == "named":
            a = self.aliases.get((t[1], t[2]))
            return self.canon(a, depth + 1) if a is not None else t
        if k in ("ptr", "slice", "array", "chan", "typeval"):
            return (k, self.canon(t[1], depth + 1))
        if k == "map":
            return (k, self.canon(t[1], depth + 1), self.canon(t[2], depth + 1))
        if k == "func":
            return (k, tuple(self.canon(x, depth + 1) for x in t[1]), tuple(self.canon(x, depth + 1) for x in t[2]), t[3])
        if k == "struct":
            return (k, tuple((n, self.canon(x, depth + 1), e) for n, x, e in t[1]))
        if k == "iface":
            return (k, {n: (self.canon(ft, depth + 1), p) for n, (ft, p) in t[1].items()},
                    tuple(self.canon(e, depth + 1) for e in t[2]))
        return t

    def finalize(self):
        """Resolve aliases through every stored declaration (they may be declared in any file)."""
        self.types = {k: self.canon(v) for k, v in self.types.items()}
        self.methods = {k: {n: (self.canon(ft), p) for n, (ft, p) in v.items()} for k, v in self.methods.items()}
        self.funcs = {k: self.canon(v) for k, v in self.funcs.items()}
        self.values = {k: (v if v[0] == "lazy" else self.canon(v)) for k, v in self.values.items()}
        for k in list(self.aliases):
            self.types[k] = self.canon(self.types[k])
        self.final = True


class FuncDecl:
    def __init__(self, name, recv, ftype, params, results, body, line, end):
        self.name, self.recv, self.ftype = name, recv, ftype
        self.params, self.results, self.body, self.line, self.end = params, results, body, line, end


class Cursor:
    def __init__(self, toks, i=0):
        self.toks, self.i = toks, i

    def peek(self, k=0):
        return self.toks[min(self.i + k, len(self.toks) - 1)]

    def next(self):
        t = self.peek()
        self.i += 1
        return t

    def at(self, text, k=0):
        return self.peek(k).text == text and self.peek(k).kind in ("op", "id")

    def accept(self, text):
        if self.at(text):
            self.i += 1
            return True
        return False

    def expect(self, text):
        t = self.next()
        if t.text != text:
            raise GoError("line %d: expected %r, got %r" % (t.line, text, t.text))
        return t

    def ident(self):
        t = self.next()
        if t.kind != "id":
            raise GoError("line %d: expected identifier, got %r" % (t.line, t.text))
        return t.text

    def skip_balanced(self):
        """At an opening bracket: move past its match."""
        pairs = {"(": ")", "[": "]", "{": "}"}
        stack = []
        while True:
            t = self.next()
            if t.kind == "eof":
                raise GoError("unbalanced brackets")
            if t.kind == "op" and t.text in pairs:
                stack.append(pairs[t.text])
            elif t.kind == "op" and stack and t.text == stack[-1]:
                stack.pop()
                if not stack:
                    return


class TypeParser:
    """Type expressions (shared by declarations and statements)."""

    def __init__(self, uni, ctx):
        self.uni, self.ctx = uni, ctx

    tparams = frozenset()

    def qualify(self, name):
        if name in self.tparams:
            return UNKNOWN   # a type parameter
        if name in BUILTIN_TYPES:
            return named("", name)
        return named(self.ctx.pkg, name)

    def parse_type(self, c):
        t = c.peek()
        if t.text == "*":
            c.next()
            return ("ptr", self.parse_type(c))
        if t.text == "(":
            c.next()
            r = self.parse_type(c)
            c.expect(")")
            return r
        if t.text == "[":
            c.next()
            if c.accept("]"):
                return ("slice", self.parse_type(c))
            while not c.at("]"):
                if c.peek().kind == "eof":
                    raise GoError("bad array type")
                c.next()
            c.expect("]")
            return ("array", self.parse_type(c))
        if t.text == "map":
            c.next()
            c.expect("[")
            k = self.parse_type(c)
            c.expect("]")
            return ("map", k, self.parse_type(c))
        if t.text == "chan":
            c.next()
            c.accept("<-")
            return ("chan", self.parse_type(c))
        if t.text == "<-":
            c.next()
            c.expect("chan")
            return ("chan", self.parse_type(c))
        if t.text == "func":
            c.next()
            return self.parse_signature(c)[0]
        if t.text == "interface":
            c.next()
            return self.parse_interface(c)
        if t.text == "struct":
            c.next()
            return self.parse_struct(c)
        if t.kind == "id":
            c.next()
            name = t.text
            if c.at(".") and name in self.ctx.imports:
                c.next()
                sel = c.ident()
                pkg = self.ctx.imports[name]
                r = named(pkg, sel)
            else:
                r = self.qualify(name)
            if c.at("[") and not c.at("]", 1):   # generic instantiation: not tracked
                c.skip_balanced()
                return UNKNOWN
            return self.uni.canon(r) if self.uni.final else r
        raise GoError("line %d: expected type, got %r" % (t.line, t.text))

    def parse_params(self, c):
        """'(' params ')' -> [(name or None, type)], variadic."""
        c.expect("(")
        groups = []   # list of token spans per comma-separated item
        cur, depth = [], 0
        while True:
            t = c.next()
            if t.kind == "eof":
                raise GoError("unterminated parameters")
            if depth == 0 and t.text in (",", ")"):
                if cur:
                    groups.append(cur)
                cur = []
                if t.text == ")":
                    break
                continue
            if t.text in ("(", "[", "{"):
                depth += 1
            elif t.text in (")", "]", "}"):
                depth -= 1
            cur.append(t)
        named_form = any(len(g) >= 2 and g[0].kind == "id" and g[0].text not in KEYWORDS
                         and g[1].text != "." for g in groups)
        out, variadic, pending = [], False, []
        for g in groups:
            if named_form:
                if len(g) == 1:
                    pending.append(g[0].text)
                    continue
                name, rest = g[0].text, g[1:]
            else:
                name, rest = None, g
            if rest and rest[0].text == "...":
                variadic = True
                rest = rest[1:]
                ty = ("slice", self.parse_type(Cursor(rest + [Tok("eof", "", 0)])))
            else:
                ty = self.parse_type(Cursor(rest + [Tok("eof", "", 0)]))
            for p in pending:
                out.append((p, ty))
            pending = []
            out.append((name, ty))
        for p in pending:   # unnamed single-token types
            out.append((None, self.qualify(p) if p not in self.ctx.imports else UNKNOWN))
        return out, variadic

    def parse_signature(self, c):
        params, variadic = self.parse_params(c)
        results = []
        if c.at("("):
            results, _ = self.parse_params(c)
        elif not (c.at("{") or c.at(";") or c.at(")") or c.at(",") or c.at("]") or c.at("}")
                  or c.at("=") or c.peek().kind in ("eof", "str")):
            results = [(None, self.parse_type(c))]
        ft = ("func", tuple(t for _, t in params), tuple(t for _, t in results), variadic)
        return ft, params, results

    def parse_struct(self, c):
        c.expect("{")
        fields = []
        while not c.at("}"):
            if c.accept(";"):
                continue
            start = c.i
            line = []
            while not (c.at(";") or c.at("}")):
                if c.peek().text in ("(", "[", "{"):
                    s = c.i
                    c.skip_balanced()
                    line.extend(c.toks[s:c.i])
                else:
                    line.append(c.next())
            line = [t for t in line if t.kind != "str"]   # tags
            if not line:
                continue
            sub = Cursor(line + [Tok("eof", "", 0)])
            if line[0].text == "*" or (len(line) >= 3 and line[1].text == ".") or len(line) == 1:
                ty = self.parse_type(sub)                 # embedded field
                base = ty[1] if ty[0] == "ptr" else ty
                fields.append((base[2] if base[0] == "named" else "?", ty, True))
                continue
            names = [sub.ident()]
            while sub.accept(","):
                names.append(sub.ident())
            ty = self.parse_type(sub)
            for nm in names:
                fields.append((nm, ty, False))
            del start
        c.expect("}")
        return ("struct", tuple(fields))

    def parse_interface(self, c):
        c.expect("{")
        methods, embeds = {}, []
        while not c.at("}"):
            if c.accept(";"):
                continue
            if c.peek().kind == "id" and c.at("(", 1):
                name = c.ident()
                ft = self.parse_signature(c)[0]
                methods[name] = (ft, False)
            else:
                embeds.append(self.parse_type(c))
                while not (c.at(";") or c.at("}")):   # type unions in constraints
                    c.next()
        c.expect("}")
        return ("iface", methods, tuple(embeds))


class DeclParser(TypeParser):
    """Top-level declarations of one file; function bodies are kept as token spans."""

    def __init__(self, uni, path, toks, check):
        self.uni, self.path, self.c, self.check = uni, path, Cursor(toks), check
        self.ctx = None

    def parse_file(self):
        c = self.c
        c.expect("package")
        pkg = c.ident()
        c.accept(";")
        self.ctx = FileCtx(self.path, pkg, {})
        while c.at("import"):
            c.next()
            if c.accept("("):
                while not c.accept(")"):
                    if c.accept(";"):
                        continue
                    self._import_spec()
            else:
                self._import_spec()
            c.accept(";")
        while c.peek().kind != "eof":
            t = c.peek()
            if t.text == ";":
                c.next()
            elif t.text == "func":
                self._func()
            elif t.text in ("type", "var", "const"):
                c.next()
                kind = t.text
                if c.accept("("):
                    prev = None
                    iota_i = 0
                    while not c.accept(")"):
                        if c.accept(";"):
                            continue
                        prev = self._spec(kind, prev, iota_i)
                        iota_i += 1
                else:
                    self._spec(kind, None, 0)
            else:
                raise GoError("%s:%d: unexpected %r at top level" % (self.path, t.line, t.text))

    def _import_spec(self):
        c = self.c
        alias = None
        if c.peek().kind == "id" or c.at(".") or c.at("_"):
            alias = c.next().text
        path = c.next().text.strip('"`')
        if alias in (None,):
            alias = path.rsplit("/", 1)[-1]
        pkg = "C" if path == "C" else path.rsplit("/", 1)[-1]
        self.ctx.imports[alias] = pkg

    def _site(self, name, line):
        self.uni.decl_sites.setdefault((self.ctx.pkg, name), []).append("%s:%d" % (os.path.basename(self.path), line))

    def _spec(self, kind, prev, iota_i):
        c = self.c
        line = c.peek().line
        if kind == "type":
            name = c.ident()
            if c.at("[") and not c.at("]", 1):
                c.skip_balanced()   # type parameters
            alias = c.accept("=")
            ty = self.parse_type(c)
            if alias:
                self.uni.aliases[(self.ctx.pkg, name)] = ty
            self.uni.types[(self.ctx.pkg, name)] = ty
            self._site(name, line)
            return None
        names = [c.ident()]
        while c.accept(","):
            names.append(c.ident())
        ty = None
        if not (c.at("=") or c.at(";") or c.at(")")):
            ty = self.parse_type(c)
        value = None
        if c.accept("="):
            start = c.i
            depth = 0
            while True:
                t = c.peek()
                if t.kind == "eof":
                    break
                if depth == 0 and t.text in (";", ")"):
                    break
                if t.text in ("(", "[", "{"):
                    depth += 1
                elif t.text in (")", "]", "}"):
                    depth -= 1
                c.next()
            value = c.toks[start:c.i]
        if kind == "const" and ty is None and value is None and prev is not None:
            ty, value = prev
        for nm in names:
            if nm == "_":
                if self.check is True and ty is not None and value:
                    self.uni.assertions.append((self.ctx, ty, value, line))
                continue
            if ty is not None:
                self.uni.values[(self.ctx.pkg, nm)] = ty
            elif value:
                self.uni.values[(self.ctx.pkg, nm)] = ("lazy", value, self.ctx)
            else:
                self.uni.values[(self.ctx.pkg, nm)] = UNKNOWN
            self._site(nm, line)
        return (ty, value)

    def _func(self):
        c = self.c
        line = c.next().line
        recv = None
        rparams = []
        rtp = frozenset()
        if c.at("("):
            s0 = c.i
            c.skip_balanced()
            rt = c.toks[s0:c.i]
            c.i = s0
            # type parameters of a generic receiver (m *T[K, V]): the names inside its brackets
            if any(t.text == "[" for t in rt):
                b0 = next(i for i, t in enumerate(rt) if t.text == "[")
                rtp = frozenset(t.text for t in rt[b0:] if t.kind == "id")
            rparams, _ = self.parse_params(c)
            rt = rparams[0][1] if rparams else UNKNOWN
            ptr = rt[0] == "ptr"
            base = rt[1] if ptr else rt
            recv = (base, ptr)
        name = c.ident()
        self.tparams = rtp
        if c.at("["):   # type parameters: unknown types inside the signature and the body
            s0 = c.i
            c.skip_balanced()
            tp = c.toks[s0:c.i]
            self.tparams = rtp | frozenset(tp[i].text for i in range(1, len(tp) - 1)
                                           if tp[i].kind == "id" and tp[i - 1].text in ("[", ","))
        ft, params, results = self.parse_signature(c)
        body = None
        if c.at("{"):
            s = c.i
            c.skip_balanced()
            body = (s, c.i)
        if recv is not None:
            base, ptr = recv
            if base[0] == "named":
                self.uni.methods.setdefault((base[1], base[2]), {})[name] = (ft, ptr)
        elif name not in ("init", "_"):
            self.uni.funcs[(self.ctx.pkg, name)] = ft
            self._site(name, line)
        if self.check and body is not None:
            end = c.toks[body[1] - 1].line
            if self.check is True or any(line <= ln <= end for ln in self.check):
                fd = FuncDecl(name, (rparams[0] if rparams else None), ft, params, results,
                              Cursor(c.toks, body[0]), line, end)
                fd.tparams = self.tparams
                self.uni.bodies.append((self.ctx, fd))
        self.tparams = frozenset()


Universe.assertions = None  # set per instance in load_universe


# ----------------------------------------------------------------------------- checking

STDLIB = {
    ("fmt", "Errorf"): ("func", (named("", "string"), ("slice", named("", "any"))), (named("", "error"),), True),
    ("fmt", "Sprintf"): ("func", (named("", "string"), ("slice", named("", "any"))), (named("", "string"),), True),
    ("errors", "New"): ("func", (named("", "string"),), (named("", "error"),), False),
    ("os", "Getenv"): ("func", (named("", "string"),), (named("", "string"),), False),
    ("strconv", "Atoi"): ("func", (named("", "string"),), (named("", "int"), named("", "error")), False),
    ("runtime", "LockOSThread"): ("func", (), (), False),
    ("runtime", "UnlockOSThread"): ("func", (), (), False),
    ("C", "GoString"): ("func", (("ptr", named("C", "char")),), (named("", "string"),), False),
    ("C", "malloc"): ("func", (named("C", "size_t"),), (named("unsafe", "Pointer"),), False),
    ("C", "free"): ("func", (named("unsafe", "Pointer"),), (), False),
}
STDLIB_TYPES = {("unsafe", "Pointer"), ("runtime", "Pinner"), ("sync", "Once"), ("sync", "Mutex"),
                ("sync", "Pool"), ("sync", "RWMutex"), ("bytes", "Reader"), ("io", "Reader")}


class Var:
    __slots__ = ("name", "t", "local", "line", "used")

    def __init__(self, name, t, local, line):
        self.name, self.t, self.local, self.line, self.used = name, t, local, line, False


ASSIGN_OPS = {"=", "+=", "-=", "*=", "/=", "%=", "&=", "|=", "^=", "<<=", ">>=", "&^=", "++", "--", ","}


class Checker:
    def __init__(self, uni):
        if not uni.final:
            uni.finalize()
        self.uni = uni
        self.tparams = frozenset()
        self.errors = []
        self.stats = {"selectors": 0, "selectors_typed": 0, "calls": 0, "calls_typed": 0,
                      "c_args": 0, "c_args_typed": 0, "idents": 0, "assigns_typed": 0, "stmts": 0}
        self.ctx = None
        self.scopes = []
        self.results = []
        self.lhs_mode = False   # parsing the left side of an assignment: a bare name there is not a use
        self.breaks = []        # per enclosing for / switch / select: [saw a break]; None: a function boundary

    def tp(self):
        t = TypeParser(self.uni, self.ctx)
        t.tparams = self.tparams
        return t

    def err(self, line, msg):
        self.errors.append("%s:%d: %s" % (os.path.basename(self.ctx.path), line, msg))

    # ---- scopes
    def push(self):
        self.scopes.append({})

    def pop(self):
        for v in self.scopes.pop().values():
            if v.local and not v.used:
                self.err(v.line, "declared and not used: %s" % v.name)

    def declare(self, name, t, local=False, line=0):
        """local: a variable of := / var / range, which Go requires to be read somewhere."""
        if name != "_":
            self.scopes[-1][name] = Var(name, t, local, line)

    def lookup_local(self, name):
        for s in reversed(self.scopes):
            if name in s:
                return s[name]
        return None

    # ---- type helpers
    def value_of(self, pkg, name):
        v = self.uni.values.get((pkg, name))
        if v is not None and v[0] == "lazy":
            self.uni.values[(pkg, name)] = UNKNOWN   # cycle guard
            saved = (self.ctx, self.scopes)
            self.ctx, self.scopes = v[2], [{}]
            try:
                t = self.expr(Cursor(list(v[1]) + [Tok("eof", "", 0)]))
            except GoError:
                t = UNKNOWN
            self.ctx, self.scopes = saved
            if t[0] == "tuple":
                t = UNKNOWN
            self.uni.values[(pkg, name)] = t
            return t
        return v

    def is_iface(self, t):
        return self.uni.underlying(t)[0] == "iface"

    def is_numeric(self, t):
        u = self.uni.underlying(t)
        if u[0] == "named" and u[1] == "" and (u[2] in INT_NAMES or u[2] in FLOAT_NAMES):
            return True
        return u[0] == "named" and u[1] == "C" and (u[2] in C_NUMERIC or u[2] in INT_NAMES)

    def identical(self, a, b):
        if a == UNKNOWN or b == UNKNOWN or a[0] == "?" or b[0] == "?":
            return True
        if (a[0] == "named" and not self.known(a)) or (b[0] == "named" and not self.known(b)):
            return True   # a type parameter, or a type of a package not loaded
        if a[0] != b[0]:
            return False
        k = a[0]
        if k == "named":
            return a[1:] == b[1:]
        if k in ("ptr", "slice", "array", "chan"):
            return self.identical(a[1], b[1])
        if k == "map":
            return self.identical(a[1], b[1]) and self.identical(a[2], b[2])
        if k == "func":
            return (len(a[1]) == len(b[1]) and len(a[2]) == len(b[2]) and a[3] == b[3]
                    and all(self.identical(x, y) for x, y in zip(a[1], b[1]))
                    and all(self.identical(x, y) for x, y in zip(a[2], b[2])))
        return a == b

    def known(self, t):
        """A type every part of which is loaded (so a mismatch is a real one)."""
        k = t[0]
        if k == "named":
            if t[1] in ("", "C", "unsafe"):
                return True
            return self.uni.is_loaded(t[1]) and (t[1], t[2]) in self.uni.types
        if k in ("ptr", "slice", "array", "chan"):
            return self.known(t[1])
        if k == "map":
            return self.known(t[1]) and self.known(t[2])
        if k == "func":
            return all(self.known(x) for x in t[1] + t[2])
        return k == "untyped"

    def assignable(self, v, t):
        if v == UNKNOWN or t == UNKNOWN or v[0] in ("?", "tuple") or not self.known(t) or not self.known(v):
            return True
        if v[0] == "untyped":
            kind = v[1]
            u = self.uni.underlying(t)
            if u[0] == "iface" or u == UNKNOWN:
                return True
            if kind == "nil":
                return u[0] in ("ptr", "slice", "map", "chan", "func") or t == named("unsafe", "Pointer")
            if kind in ("int", "rune"):
                return self.is_numeric(t)
            if kind == "float":
                return self.is_numeric(t)
            if kind == "string":
                return u == named("", "string")
            if kind == "bool":
                return u == named("", "bool")
            return True
        if self.identical(v, t):
            return True
        if self.is_iface(t):
            return self.implements(v, t) is None
        # identical underlying types where one side is unnamed
        if (v[0] != "named" or t[0] != "named") and self.identical(self.uni.underlying(v), self.uni.underlying(t)):
            return True
        return False

    def method_set(self, t):
        """name -> functype of the methods callable on a value of type t (promotion included)."""
        out = {}
        ptr = t[0] == "ptr"
        base = t[1] if ptr else t
        self._collect_methods(base, ptr, out, 0)
        return out

    def _collect_methods(self, base, ptr, out, depth):
        if depth > 5 or base[0] != "named":
            return
        for name, (ft, precv) in self.uni.methods.get((base[1], base[2]), {}).items():
            if name not in out and (ptr or not precv):
                out[name] = ft
        u = self.uni.underlying(base)
        if u[0] == "iface":
            for name, ft in self.iface_methods(u).items():
                out.setdefault(name, ft)
        if u[0] == "struct":
            for fname, fty, emb in u[1]:
                if emb:
                    eptr = fty[0] == "ptr"
                    eb = fty[1] if eptr else fty
                    self._collect_methods(eb, eptr or ptr, out, depth + 1)

    def unknown_embed(self, base, depth):
        """base (a struct, through embedded fields) embeds a type whose methods are not known."""
        if depth > 5 or base[0] != "named":
            return False
        u = self.uni.underlying(base)
        if u[0] == "iface":
            return any(self.uni.underlying(e) == UNKNOWN for e in u[2])
        if u[0] != "struct":
            return False
        for _, fty, emb in u[1]:
            if emb:
                eb = fty[1] if fty[0] == "ptr" else fty
                if self.uni.underlying(eb) == UNKNOWN or self.unknown_embed(eb, depth + 1):
                    return True
        return False

    def iface_methods(self, u, depth=0):
        out = {name: ft for name, (ft, _) in u[1].items()}
        for e in u[2]:
            eu = self.uni.underlying(e)
            if eu[0] == "iface" and depth < 5:
                for name, ft in self.iface_methods(eu, depth + 1).items():
                    out.setdefault(name, ft)
        return out

    def implements(self, v, iface):
        """None when v's method set has every method of iface with an identical signature,
        else a message; unknown types pass."""
        base = v[1] if v[0] == "ptr" else v
        if base[0] != "named" or not self.uni.is_loaded(base[1]) or base[1] in ("", "C"):
            return None
        if self.is_iface(v):
            return None
        ms = self.method_set(v)
        for name, ft in self.iface_methods(self.uni.underlying(iface)).items():
            if name not in ms:
                if self.unknown_embed(base, 0):
                    return None   # maybe promoted from an embedded type of a package not loaded
                return "%s does not implement %s (missing method %s)" % (fmt_type(v), fmt_type(iface), name)
            if not self.identical(ms[name], ft):
                return "%s does not implement %s (method %s has type %s, want %s)" % (
                    fmt_type(v), fmt_type(iface), name, fmt_type(ms[name]), fmt_type(ft))
        return None

    def select(self, t, name, line):
        """Type of x.name for x of type t (a field or a method value)."""
        self.stats["selectors"] += 1
        if t == UNKNOWN or t[0] in ("?", "untyped", "tuple"):
            return UNKNOWN
        ptr = t[0] == "ptr"
        base = t[1] if ptr else t
        if base[0] != "named":
            if base[0] == "struct":
                for fname, fty, _ in base[1]:
                    if fname == name:
                        self.stats["selectors_typed"] += 1
                        return fty
            return UNKNOWN
        if base[1] not in ("",) and not self.uni.is_loaded(base[1]):
            return UNKNOWN
        found = self._lookup(base, name, 0)
        if found == UNKNOWN:
            return UNKNOWN
        if found is None:
            if self.uni.underlying(base) == UNKNOWN:
                return UNKNOWN
            self.err(line, "%s has no field or method %s" % (fmt_type(t), name))
            return UNKNOWN
        self.stats["selectors_typed"] += 1
        return found

    def _lookup(self, base, name, depth):
        if depth > 5 or base[0] != "named":
            return None
        m = self.uni.methods.get((base[1], base[2]), {})
        if name in m:
            return m[name][0]
        u = self.uni.underlying(base)
        if u[0] == "iface":
            r = self.iface_methods(u).get(name)
            if r is None and any(self.uni.underlying(e) == UNKNOWN for e in u[2]):
                return UNKNOWN   # maybe from an embedded interface of an unloaded package
            return r
        if u[0] == "struct":
            for fname, fty, emb in u[1]:
                if fname == name:
                    return fty
            maybe = False
            for fname, fty, emb in u[1]:
                if emb:
                    eb = fty[1] if fty[0] == "ptr" else fty
                    r = self._lookup(eb, name, depth + 1)
                    if r == UNKNOWN or (r is None and self.uni.underlying(eb) == UNKNOWN):
                        maybe = True
                    elif r is not None:
                        return r
            if maybe:
                return UNKNOWN
        return None

    # ---- expressions
    PREC = {"||": 1, "&&": 2, "==": 3, "!=": 3, "<": 3, "<=": 3, ">": 3, ">=": 3,
            "+": 4, "-": 4, "|": 4, "^": 4, "*": 5, "/": 5, "%": 5, "<<": 5, ">>": 5, "&": 5, "&^": 5}

    def expr(self, c, nocomp=False):
        return self.binary(c, 1, nocomp)

    def binary(self, c, minp, nocomp):
        left = self.unary(c, nocomp)
        while True:
            t = c.peek()
            p = self.PREC.get(t.text) if t.kind == "op" else None
            if p is None or p < minp:
                return left
            c.next()
            right = self.binary(c, p + 1, nocomp)
            left = self.binop(t.text, left, right, t.line)

    def binop(self, op, a, b, line):
        if op in ("&&", "||"):
            return untyped("bool")
        if op in ("<<", ">>"):
            return a
        for x in (a, b):
            if x[0] == "typeval":
                self.err(line, "type %s used as a value" % fmt_type(x[1]))
                return UNKNOWN
        cmp_ = op in ("==", "!=", "<", "<=", ">", ">=")
        if a[0] == "untyped" and b[0] == "untyped":
            if cmp_:
                return untyped("bool")
            return untyped("float" if "float" in (a[1], b[1]) else a[1])
        if a[0] == "untyped" or b[0] == "untyped":
            typed, un = (b, a) if a[0] == "untyped" else (a, b)
            if not self.assignable(un, typed):
                self.err(line, "mismatched types %s and %s (operator %s)" % (fmt_type(a), fmt_type(b), op))
            return untyped("bool") if cmp_ else typed
        if a != UNKNOWN and b != UNKNOWN and self.known(a) and self.known(b) and not self.identical(a, b):
            if not (cmp_ and (self.is_iface(a) or self.is_iface(b))):
                self.err(line, "mismatched types %s and %s (operator %s)" % (fmt_type(a), fmt_type(b), op))
        return untyped("bool") if cmp_ else a

    def unary(self, c, nocomp):
        t = c.peek()
        if t.kind == "op" and t.text in ("-", "+", "!", "^", "*", "&", "<-"):
            c.next()
            x = self.unary(c, nocomp)
            if t.text == "&":
                return ("ptr", x) if x != UNKNOWN and x[0] not in ("typeval",) else UNKNOWN
            if t.text == "*":
                if x[0] == "typeval":
                    return ("typeval", ("ptr", x[1]))
                if x[0] == "ptr":
                    return x[1]
                if x != UNKNOWN and x[0] != "?" and self.known(x):
                    self.err(t.line, "invalid indirect of %s" % fmt_type(x))
                return UNKNOWN
            if t.text == "!":
                return untyped("bool") if x[0] == "untyped" else (x if x != UNKNOWN else UNKNOWN)
            if t.text == "<-":
                u = self.uni.underlying(x) if x != UNKNOWN and x[0] != "?" else UNKNOWN
                return ("assert", u[1]) if u[0] == "chan" else UNKNOWN
            return x
        return self.primary(c, nocomp)

    def operand(self, c, nocomp):
        t = c.next()
        if t.kind == "num":
            return untyped("float" if re.search(r"[.eE]", t.text) and not t.text.lower().startswith("0x") else "int")
        if t.kind == "str":
            return untyped("string")
        if t.kind == "rune":
            return untyped("rune")
        if t.text == "(":
            x = self.nested(lambda: self.expr(c))
            c.expect(")")
            return x
        if t.text in ("[", "map", "chan", "struct", "interface"):
            c.i -= 1
            return ("typeval", self.tp().parse_type(c))
        if t.text == "func":
            ft, params, results = self.tp().parse_signature(c)
            if c.at("{"):
                self.func_body(c, params, results, None)
                return ft
            return ("typeval", ft)
        if t.kind != "id":
            raise GoError("line %d: unexpected %r in expression" % (t.line, t.text))
        self.stats["idents"] += 1
        name = t.text
        if name == "_":
            return UNKNOWN
        if name in self.tparams:
            return ("typeval", UNKNOWN)
        loc = self.lookup_local(name)
        if loc is not None:
            if not (self.lhs_mode and c.peek().text in ASSIGN_OPS):
                loc.used = True
            return loc.t
        pkg = self.ctx.pkg
        if (pkg, name) in self.uni.types:
            return ("typeval", self.uni.canon(named(pkg, name)))
        if (pkg, name) in self.uni.funcs:
            return self.uni.funcs[(pkg, name)]
        if (pkg, name) in self.uni.values:
            return self.value_of(pkg, name)
        if name in self.ctx.imports:
            ipkg = self.ctx.imports[name]
            c.expect(".")
            sel = c.ident()
            r = self.qualified(ipkg, sel, t.line)
            if r == UNKNOWN and not self.uni.is_loaded(ipkg) and c.at("{") and not nocomp:
                self.composite(c, UNKNOWN)   # a literal of a type from an unloaded package
            return r
        if name in BUILTIN_TYPES:
            return ("typeval", named("", name))
        if name in BUILTIN_FUNCS:
            return ("builtin", name)
        if name in ("true", "false"):
            return untyped("bool")
        if name == "nil":
            return untyped("nil")
        if name == "iota":
            return untyped("int")
        self.err(t.line, "undefined: %s" % name)
        return UNKNOWN

    def qualified(self, pkg, sel, line):
        if pkg == "C":
            self.stats["idents"] += 1
            if sel in self.uni.cfuncs:
                return ("cfunc", sel)
            if sel in self.uni.cmacros:
                return untyped("int")
            if sel in self.uni.ctypes or sel in C_NUMERIC:
                return ("typeval", named("C", sel))
            if (pkg, sel) in STDLIB:
                return STDLIB[(pkg, sel)]
            self.err(line, "C.%s is not declared by the included headers" % sel)
            return UNKNOWN
        if (pkg, sel) in STDLIB:
            return STDLIB[(pkg, sel)]
        if (pkg, sel) in STDLIB_TYPES:
            return ("typeval", named(pkg, sel))
        if pkg == "unsafe" and sel in ("Slice", "SliceData", "Add", "String", "StringData", "Sizeof"):
            return ("unsafe", sel)
        if not self.uni.is_loaded(pkg):
            return UNKNOWN
        if (pkg, sel) in self.uni.types:
            return ("typeval", self.uni.canon(named(pkg, sel)))
        if (pkg, sel) in self.uni.funcs:
            return self.uni.funcs[(pkg, sel)]
        if (pkg, sel) in self.uni.values:
            return self.value_of(pkg, sel)
        if not sel[:1].isupper():
            self.err(line, "%s.%s is not exported" % (pkg, sel))
        else:
            self.err(line, "undefined: %s.%s" % (pkg, sel))
        return UNKNOWN

    def primary(self, c, nocomp):
        x = self.operand(c, nocomp)
        while True:
            t = c.peek()
            if t.text == "." and t.kind == "op":
                c.next()
                if c.accept("("):
                    if c.accept("type"):
                        c.expect(")")
                        x = UNKNOWN
                        continue
                    ty = self.tp().parse_type(c)
                    c.expect(")")
                    x = ("assert", ty)
                    continue
                name = c.ident()
                if x[0] == "typeval":   # method expression (*T).M
                    mt = self.select(x[1], name, t.line)
                    x = ("func", (x[1],) + mt[1], mt[2], mt[3]) if mt[0] == "func" else UNKNOWN
                else:
                    x = self.select(self.strip_assert(x), name, t.line)
            elif t.text == "[" and t.kind == "op":
                c.next()
                x = self.nested(lambda: self.index(c, self.strip_assert(x), t.line))
            elif t.text == "(" and t.kind == "op":
                c.next()
                x = self.nested(lambda: self.call(c, x, t.line))
            elif t.text == "{" and t.kind == "op" and x[0] == "typeval" and not nocomp:
                x = self.nested(lambda: self.composite(c, x[1]))
            else:
                return x

    def nested(self, fn):
        """Parse inside brackets: names there are read, even on an assignment's left side."""
        saved, self.lhs_mode = self.lhs_mode, False
        try:
            return fn()
        finally:
            self.lhs_mode = saved

    @staticmethod
    def strip_assert(x):
        """The value of a map index or type assertion (their comma-ok forms are the statements')."""
        return x[1] if x[0] in ("assert", "mapindex") else x

    def index(self, c, x, line):
        # slice expression or index
        lo = None
        if not c.at(":"):
            lo = self.expr(c)
        if c.accept(":"):
            if not c.at("]"):
                self.expr(c)
            if c.accept(":"):
                self.expr(c)
            c.expect("]")
            u = self.uni.underlying(x) if x != UNKNOWN else UNKNOWN
            if u[0] == "array":
                return ("slice", u[1])
            if u[0] == "ptr" and self.uni.underlying(u[1])[0] == "array":
                return ("slice", self.uni.underlying(u[1])[1])
            return x
        c.expect("]")
        if x == UNKNOWN or x[0] in ("?",):
            return UNKNOWN
        if x[0] == "typeval":
            return ("typeval", UNKNOWN)   # generic instantiation: a type, possibly of a composite literal
        u = self.uni.underlying(x)
        if u[0] == "map":
            if lo is not None and not self.assignable(lo, u[1]):
                self.err(line, "cannot use %s as %s map key" % (fmt_type(lo), fmt_type(u[1])))
            return ("mapindex", u[2])
        if u[0] in ("slice", "array"):
            return u[1]
        if u[0] == "ptr" and self.uni.underlying(u[1])[0] == "array":
            return self.uni.underlying(u[1])[1]
        if u == named("", "string"):
            return named("", "uint8")
        if u == UNKNOWN:
            return UNKNOWN
        if self.known(x):
            self.err(line, "cannot index %s" % fmt_type(x))
        return UNKNOWN

    def args(self, c):
        out, spread = [], False
        while not c.at(")"):
            a = self.expr(c)
            if a[0] == "mapindex":
                a = a[1]
            out.append(self.strip_assert(a))
            if c.accept("..."):
                spread = True
            if not c.accept(","):
                break
        c.expect(")")
        return out, spread

    def call(self, c, f, line):
        self.stats["calls"] += 1
        f = self.strip_assert(f)
        if f[0] == "builtin":
            self.stats["calls_typed"] += 1
            return self.builtin(c, f[1], line)
        if f[0] == "typeval":   # conversion
            args, _ = self.args(c)
            if len(args) != 1:
                self.err(line, "conversion to %s takes one argument" % fmt_type(f[1]))
            self.stats["calls_typed"] += 1
            return f[1]
        if f[0] == "unsafe":
            args, _ = self.args(c)
            a0 = args[0] if args else UNKNOWN
            self.stats["calls_typed"] += 1
            if f[1] == "Slice":
                return ("slice", a0[1]) if a0[0] == "ptr" else UNKNOWN
            if f[1] == "SliceData":
                u = self.uni.underlying(a0) if a0 != UNKNOWN else UNKNOWN
                return ("ptr", u[1]) if u[0] == "slice" else UNKNOWN
            if f[1] == "Add":
                return named("unsafe", "Pointer")
            if f[1] == "Sizeof":
                return named("", "uintptr")
            return UNKNOWN
        cname = None
        if f[0] == "cfunc":
            cname = f[1]
            f = self.uni.cfuncs[cname]
        args, spread = self.args(c)
        if f[0] != "func":
            return UNKNOWN
        self.stats["calls_typed"] += 1
        params, results, variadic = f[1], f[2], f[3]
        if len(args) == 1 and args[0][0] == "tuple" and len(args[0][1]) > 1:
            args = list(args[0][1])
        n = len(params)
        if variadic and not spread:
            ok = len(args) >= n - 1
        else:
            ok = len(args) == n
        if not ok:
            self.err(line, "%s: %d arguments, want %d" % (("C." + cname) if cname else "call", len(args), n))
        else:
            for i, a in enumerate(args):
                if variadic and not spread and i >= n - 1:
                    pt = params[-1][1] if params[-1][0] == "slice" else UNKNOWN
                else:
                    pt = params[i]
                if cname:
                    self.stats["c_args"] += 1
                    if a != UNKNOWN and a[0] != "?":
                        self.stats["c_args_typed"] += 1
                if not self.assignable(a, pt):
                    self.err(line, "%sargument %d: cannot use %s as %s" % (
                        ("C.%s " % cname) if cname else "", i + 1, fmt_type(a), fmt_type(pt)))
        if not results:
            return ("tuple", ())
        if len(results) == 1:
            return results[0]
        return ("tuple", tuple(results))

    def builtin(self, c, name, line):
        if name in ("make", "new"):
            ty = self.tp().parse_type(c)
            while c.accept(","):
                if c.at(")"):
                    break
                self.expr(c)
            c.expect(")")
            return ty if name == "make" else ("ptr", ty)
        args, spread = self.args(c)
        if name in ("len", "cap", "copy"):
            return named("", "int")
        if name == "append":
            if args and args[0][0] not in ("untyped",):
                u = self.uni.underlying(args[0]) if args[0] != UNKNOWN else UNKNOWN
                if u[0] == "slice" and not spread and len(args) > 1:
                    for a in args[1:]:
                        if not self.assignable(a, u[1]):
                            self.err(line, "append: cannot use %s as %s" % (fmt_type(a), fmt_type(u[1])))
                return args[0]
            return UNKNOWN
        if name in ("min", "max"):
            for a in args:
                if a[0] != "untyped":
                    return a
            return args[0] if args else UNKNOWN
        if name == "recover":
            return named("", "any")
        return ("tuple", ())

    def composite(self, c, ty):
        c.expect("{")
        u = self.uni.underlying(ty) if ty != UNKNOWN else UNKNOWN
        if u[0] == "ptr":   # &T elided in []*T{{...}}
            u = self.uni.underlying(u[1])
        while not c.at("}"):
            if c.accept(";"):
                continue
            line = c.peek().line
            if u[0] not in ("struct", "map") and c.peek().kind == "id" and c.at(":", 1):
                c.next()   # a field key of a type not loaded
                c.next()
                self.elem(c, UNKNOWN)
            elif u[0] == "struct" and c.peek().kind == "id" and c.at(":", 1):
                fname = c.ident()
                c.expect(":")
                ft = None
                for n, t, _ in u[1]:
                    if n == fname:
                        ft = t
                if ft is None:
                    self.err(line, "unknown field %s in struct literal of type %s" % (fname, fmt_type(ty)))
                    ft = UNKNOWN
                v = self.elem(c, ft)
                if not self.assignable(v, ft):
                    self.err(line, "cannot use %s as %s value in struct literal" % (fmt_type(v), fmt_type(ft)))
            else:
                et = UNKNOWN
                if u[0] in ("slice", "array"):
                    et = u[1]
                elif u[0] == "map":
                    k = self.elem(c, u[1])
                    c.expect(":")
                    et = u[2]
                    del k
                v = self.elem(c, et)
                if u[0] in ("slice", "array", "map") and not self.assignable(v, et):
                    self.err(line, "cannot use %s as %s element" % (fmt_type(v), fmt_type(et)))
            c.accept(",")
            c.accept(";")
        c.expect("}")
        return ty

    def elem(self, c, et):
        if c.at("{"):
            return self.composite(c, et)
        if c.at("&") and c.at("{", 1):
            c.next()
            return ("ptr", self.composite(c, et[1] if et[0] == "ptr" else et))
        v = self.expr(c)
        return v[1] if v[0] == "mapindex" else self.strip_assert(v)

    # ---- statements
    def func_body(self, c, params, results, recv):
        self.push()
        if recv is not None and recv[0]:
            self.declare(recv[0], recv[1])
        for n, t in params:
            if n:
                self.declare(n, t)
        for n, t in results:
            if n:
                self.declare(n, t)
        self.results.append(results)
        self.breaks.append(None)   # a function literal's body is no loop of the enclosing function
        line = c.peek().line
        term = self.block(c)
        self.breaks.pop()
        if results and not term:
            self.err(line, "missing return")
        self.results.pop()
        self.pop()

    def block(self, c):
        """Returns whether the block is a terminating statement (its last statement is)."""
        c.expect("{")
        self.push()
        term = False
        while not c.at("}"):
            if c.peek().kind == "eof":
                raise GoError("unterminated block")
            if c.at(";"):
                c.next()
                continue
            term = self.stmt(c)
        c.expect("}")
        self.pop()
        return term

    def sync(self, c):
        depth = 0
        while True:
            t = c.peek()
            if t.kind == "eof":
                return
            if depth == 0 and t.text in (";", "}"):
                if t.text == ";":
                    c.next()
                return
            if t.text in ("(", "[", "{"):
                depth += 1
            elif t.text in (")", "]", "}"):
                depth -= 1
            c.next()

    def stmt(self, c):
        self.stats["stmts"] += 1
        start = c.i
        try:
            return bool(self._stmt(c))
        except GoError as e:
            self.err(c.toks[start].line, "cannot check statement: %s" % e)
            c.i = start
            c.next()
            self.sync(c)
            return True   # unknown: no second report

    def _end(self, c):
        if not (c.accept(";") or c.at("}")):
            t = c.peek()
            raise GoError("line %d: unexpected %r after statement" % (t.line, t.text))

    def _stmt(self, c):
        t = c.peek()
        k = t.text
        if k == ";":
            c.next()
            return
        if k == "{":
            term = self.block(c)
            c.accept(";")
            return term
        if k == "var":
            c.next()
            if c.accept("("):
                while not c.accept(")"):
                    if c.accept(";"):
                        continue
                    self.var_spec(c)
            else:
                self.var_spec(c)
            self._end(c)
            return
        if k == "const":
            c.next()
            if c.accept("("):
                while not c.accept(")"):
                    if c.accept(";"):
                        continue
                    self.var_spec(c, const=True)
            else:
                self.var_spec(c, const=True)
            self._end(c)
            return
        if k == "if":
            return self.if_stmt(c)
        if k == "for":
            return self.for_stmt(c)
        if k == "switch":
            return self.switch_stmt(c)
        if k == "select":
            return self.select_stmt(c)
        if k == "return":
            c.next()
            vals = []
            if not (c.at(";") or c.at("}")):
                vals = self.expr_list(c)
            self.check_return(vals, t.line)
            self._end(c)
            return True
        if k in ("defer", "go"):
            c.next()
            self.expr(c)
            self._end(c)
            return
        if k in ("break", "continue", "goto", "fallthrough"):
            c.next()
            labeled = c.peek().kind == "id"
            if labeled:
                c.next()
            if k == "break":   # the loop / switch it leaves is not terminating (a label: the innermost, conservatively)
                for i in range(len(self.breaks) - 1, -1, -1):
                    if self.breaks[i] is None:
                        break
                    self.breaks[i][0] = True
                    break
            self._end(c)
            return k in ("goto", "fallthrough")
        if t.kind == "id" and c.at(":", 1) and not c.at("=", 1):
            c.next()
            c.next()
            return
        is_panic = t.text == "panic" and c.at("(", 1) and self.lookup_local("panic") is None
        self.simple(c)
        self._end(c)
        return is_panic

    def expr_list(self, c, nocomp=False):
        out = [self.expr(c, nocomp)]
        while c.accept(","):
            out.append(self.expr(c, nocomp))
        return out

    def var_spec(self, c, const=False):
        names = [c.ident()]
        while c.accept(","):
            names.append(c.ident())
        ty = None
        if not (c.at("=") or c.at(";") or c.at(")") or c.at("}")):
            ty = self.tp().parse_type(c)
        vals = []
        if c.accept("="):
            vals = self.expr_list(c)
        types = self.spread(vals, len(names), c.peek().line) if vals else [ty] * len(names)
        for i, n in enumerate(names):
            vt = types[i] if i < len(types) else UNKNOWN
            if ty is not None and vals and not self.assignable(vt, ty):
                self.err(c.peek().line, "cannot use %s as %s in variable declaration" % (fmt_type(vt), fmt_type(ty)))
            if const:   # a constant keeps its untyped kind; an unused one is no error
                self.declare(n, ty if ty is not None else vt)
            else:
                self.declare(n, ty if ty is not None else self.default_type(vt), local=True, line=c.peek().line)

    def default_type(self, t):
        if t[0] == "untyped":
            return {"int": named("", "int"), "float": named("", "float64"), "rune": named("", "int32"),
                    "string": named("", "string"), "bool": named("", "bool")}.get(t[1], UNKNOWN)
        if t[0] == "mapindex":
            return t[1]
        if t[0] == "assert":
            return t[1]
        if t[0] in ("typeval", "tuple", "builtin", "cfunc", "unsafe"):
            return UNKNOWN
        return t

    def spread(self, vals, n, line, commaok=False):
        """Types for n left-hand names from a right-hand list (a tuple call spreads)."""
        if len(vals) == 1 and vals[0][0] == "tuple":
            ts = list(vals[0][1])
            if len(ts) != n and vals[0] != ("tuple", ()):
                self.err(line, "assignment mismatch: %d variables but the call returns %d values" % (n, len(ts)))
                return [UNKNOWN] * n
            if vals[0] == ("tuple", ()):
                self.err(line, "the call returns no value")
                return [UNKNOWN] * n
            return ts
        if len(vals) == 1 and n > 1 and vals[0] == UNKNOWN:   # a call into an unloaded package
            return [UNKNOWN] * n
        if len(vals) == 1 and n == 2 and vals[0][0] in ("mapindex", "assert"):
            return [vals[0][1], named("", "bool")]
        if len(vals) != n:
            self.err(line, "assignment mismatch: %d variables but %d values" % (n, len(vals)))
            return [UNKNOWN] * n
        out = []
        for v in vals:
            if v[0] == "tuple":
                self.err(line, "multiple-value call in single-value context")
                v = UNKNOWN
            out.append(v[1] if v[0] in ("mapindex", "assert") else v)
        return out

    def lhs_names(self, c):
        """Identifiers before ':=' (the cursor is at the statement start), or None."""
        i, names = c.i, []
        while True:
            t = c.toks[i]
            if t.kind != "id":
                return None
            names.append(t.text)
            nt = c.toks[i + 1]
            if nt.text == ":=":
                return names, i + 2
            if nt.text != ",":
                return None
            i += 2

    def simple(self, c, header=False):
        line = c.peek().line
        d = self.lhs_names(c)
        if d is not None:
            names, j = d
            c.i = j
            if c.accept("range"):
                x = self.expr(c, nocomp=header)
                self.range_decl(names, x, line)
                return
            vals = self.expr_list(c, nocomp=header)
            types = self.spread(vals, len(names), line)
            new = False
            for n, vt in zip(names, types):
                prev = self.scopes[-1].get(n)
                if prev is not None and n != "_":
                    if not self.assignable(vt, prev.t):
                        self.err(line, "cannot assign %s to %s (type %s)" % (fmt_type(vt), n, fmt_type(prev.t)))
                    continue
                if n != "_":
                    new = True
                self.declare(n, self.default_type(vt), local=True, line=line)
            if not new and any(n != "_" for n in names):
                self.err(line, "no new variables on left side of :=")
            return
        if c.at("range"):
            c.next()
            self.expr(c, nocomp=header)
            return
        self.lhs_mode = True
        try:
            lhs = self.expr_list(c, nocomp=header)
        finally:
            self.lhs_mode = False
        t = c.peek()
        if t.kind == "op" and (t.text == "=" or (t.text.endswith("=") and t.text not in ("==", "!=", "<=", ">=", ":="))):
            c.next()
            vals = self.expr_list(c, nocomp=header)
            if t.text == "=":
                types = self.spread(vals, len(lhs), line)
                for l_, v in zip(lhs, types):
                    lt = l_[1] if l_[0] in ("mapindex", "assert") else l_
                    if lt[0] == "typeval":
                        self.err(line, "cannot assign to a type")
                        continue
                    if lt != UNKNOWN and v != UNKNOWN:
                        self.stats["assigns_typed"] += 1
                    if not self.assignable(v, lt):
                        self.err(line, "cannot use %s as %s in assignment" % (fmt_type(v), fmt_type(lt)))
            else:
                lt = lhs[0][1] if lhs[0][0] == "mapindex" else lhs[0]
                self.binop(t.text[:-1], lt, vals[0], line)
            return
        if c.accept("++") or c.accept("--"):
            return
        if c.accept("<-"):
            self.expr(c)
            return

    def range_decl(self, names, x, line):
        x = x[1] if x[0] == "mapindex" else x
        u = self.uni.underlying(x) if x != UNKNOWN and x[0] not in ("untyped", "?") else UNKNOWN
        if x[0] == "untyped":
            kv = [named("", "int")]
        elif u[0] == "map":
            kv = [u[1], u[2]]
        elif u[0] in ("slice", "array"):
            kv = [named("", "int"), u[1]]
        elif u == named("", "string"):
            kv = [named("", "int"), named("", "int32")]
        elif u[0] == "chan":
            kv = [u[1]]
        elif u[0] == "named" and u[1] == "" and u[2] in INT_NAMES:
            kv = [x]
        else:
            kv = [UNKNOWN, UNKNOWN]
        if len(names) > len(kv):
            self.err(line, "range over %s permits only %d iteration variable(s)" % (fmt_type(x), len(kv)))
        for n, t in zip(names, kv):
            self.declare(n, t, local=True, line=line)

    def header(self, c):
        """if / switch header: [simple ';'] [expr]; the cursor stops at '{'."""
        j, depth, has_semi = c.i, 0, False
        while True:
            t = c.toks[j]
            if t.kind == "eof":
                break
            if depth == 0 and t.text == "{" and self._block_brace(c, j):
                break
            if depth == 0 and t.text == ";":
                has_semi = True
                break
            if t.text in ("(", "["):
                depth += 1
            elif t.text in (")", "]"):
                depth -= 1
            elif t.text == "{":
                depth += 1
            elif t.text == "}":
                depth -= 1
            j += 1
        if has_semi:
            self.simple(c, header=True)
            c.expect(";")
        if c.at("{"):
            return None
        if self.lhs_names(c) is not None:   # switch v := x.(type)
            self.simple(c, header=True)
            return None
        return self.expr(c, nocomp=True)

    def _block_brace(self, c, j):
        # a '{' at depth 0 in a header opens the block unless it follows a func literal signature
        prev = c.toks[j - 1]
        return not (prev.text == ")" and self._is_func_sig_end(c, j - 1))

    def _is_func_sig_end(self, c, j):
        depth = 0
        while j >= 0:
            t = c.toks[j]
            if t.text == ")":
                depth += 1
            elif t.text == "(":
                depth -= 1
                if depth == 0:
                    return j > 0 and c.toks[j - 1].text == "func"
            j -= 1
        return False

    def if_stmt(self, c):
        c.expect("if")
        self.push()
        line = c.peek().line
        cond = self.header(c)
        if cond is not None and cond != UNKNOWN and cond[0] != "?":
            u = self.uni.underlying(cond) if cond[0] != "untyped" else cond
            if u not in (named("", "bool"), untyped("bool")) and self.known(cond):
                self.err(line, "non-boolean condition in if statement (%s)" % fmt_type(cond))
        term = self.block(c)
        if c.accept("else"):
            if c.at("if"):
                t2 = self.if_stmt(c)
                self.pop()
                return term and t2
            t2 = self.block(c)
            self.pop()
            c.accept(";")
            return term and t2
        self.pop()
        c.accept(";")
        return False

    def for_stmt(self, c):
        line = c.expect("for").line
        self.push()
        forever = c.at("{")
        if not c.at("{"):
            j, depth, semis = c.i, 0, 0
            while True:
                t = c.toks[j]
                if t.kind == "eof" or (depth == 0 and t.text == "{" and self._block_brace(c, j)):
                    break
                if depth == 0 and t.text == ";":
                    semis += 1
                if t.text in ("(", "[", "{"):
                    depth += 1
                elif t.text in (")", "]", "}"):
                    depth -= 1
                j += 1
            if semis == 2:
                if not c.at(";"):
                    self.simple(c, header=True)
                c.expect(";")
                if not c.at(";"):
                    self.expr(c, nocomp=True)
                c.expect(";")
                if not c.at("{"):
                    self.simple(c, header=True)
            else:
                self.simple(c, header=True)
        del line
        self.breaks.append([False])
        self.block(c)
        broke = self.breaks.pop()[0]
        self.pop()
        c.accept(";")
        return forever and not broke

    def switch_stmt(self, c):
        c.expect("switch")
        self.push()
        tag = self.header(c)
        c.expect("{")
        has_default, all_term = False, True
        self.breaks.append([False])
        while not c.accept("}"):
            if c.accept("case"):
                vals = self.expr_list(c)
                if tag is not None:
                    for v in vals:
                        if not self.assignable(v, tag) and not self.assignable(tag, v):
                            self.err(c.peek().line, "invalid case: mismatched types %s and %s" % (fmt_type(v), fmt_type(tag)))
            else:
                c.expect("default")
                has_default = True
            c.expect(":")
            self.push()
            term = False
            while not (c.at("case") or c.at("default") or c.at("}")):
                if c.at(";"):
                    c.next()
                    continue
                term = self.stmt(c)
            all_term = all_term and term
            self.pop()
        broke = self.breaks.pop()[0]
        self.pop()
        c.accept(";")
        return has_default and all_term and not broke

    def select_stmt(self, c):
        c.expect("select")
        c.expect("{")
        all_term = True
        self.breaks.append([False])
        while not c.accept("}"):
            self.push()
            if c.accept("case"):
                self.simple(c)
            else:
                c.expect("default")
            c.expect(":")
            term = False
            while not (c.at("case") or c.at("default") or c.at("}")):
                if c.at(";"):
                    c.next()
                    continue
                term = self.stmt(c)
            all_term = all_term and term
            self.pop()
        broke = self.breaks.pop()[0]
        c.accept(";")
        return all_term and not broke

    def check_return(self, vals, line):
        want = self.results[-1] if self.results else []
        if not vals:
            if want and not all(n for n, _ in want):
                self.err(line, "not enough return values: have 0, want %d" % len(want))
            return
        types = vals
        if len(vals) == 1 and vals[0] == UNKNOWN and len(want) > 1:
            return   # a call into an unloaded package
        if len(vals) == 1 and vals[0][0] == "tuple":
            types = list(vals[0][1])
        if len(types) != len(want):
            self.err(line, "wrong number of return values: have %d, want %d" % (len(types), len(want)))
            return
        for i, (v, (_, wt)) in enumerate(zip(types, want)):
            v = v[1] if v[0] in ("mapindex", "assert") else v
            if not self.assignable(v, wt):
                self.err(line, "return value %d: cannot use %s as %s" % (i + 1, fmt_type(v), fmt_type(wt)))

    # ---- drivers
    def check_all(self):
        for ctx, fd in self.uni.bodies:
            self.ctx = ctx
            self.scopes = []
            self.tparams = getattr(fd, "tparams", frozenset())
            cn = self.uni.canon
            fd.params = [(n, cn(t)) for n, t in fd.params]
            fd.results = [(n, cn(t)) for n, t in fd.results]
            recv = fd.recv if fd.recv is None else (fd.recv[0], cn(fd.recv[1]))
            c = fd.body
            try:
                self.func_body(c, fd.params, fd.results, recv)
            except GoError as e:
                self.err(fd.line, "cannot check func %s: %s" % (fd.name, e))
        for ctx, ty, value, line in self.uni.assertions:
            self.ctx = ctx
            self.scopes = [{}]
            v = self.expr(Cursor(list(value) + [Tok("eof", "", 0)]))
            msg = self.implements(v, ty) if self.is_iface(ty) else None
            if msg:
                self.err(line, msg)
            elif not self.assignable(v, ty):
                self.err(line, "cannot use %s as %s" % (fmt_type(v), fmt_type(ty)))
        self.errors.extend(self.uni.import_errors)
        return self.errors


def load_universe(headers, packages, check_files):
    """headers: C header texts; packages: [(path, source)] loaded for declarations only;
    check_files: [(path, source)] loaded and then checked."""
    uni = Universe()
    uni.assertions = []
    for h in headers:
        uni.load_c_header(h)
    for path, src in packages:
        uni.load_go(path, src, check=False)
    for path, src in check_files:
        uni.load_go(path, src, check=True)
    uni.finalize()
    return uni


GOOS_SUFFIXES = ("aix", "android", "darwin", "dragonfly", "freebsd", "illumos", "ios", "js", "linux", "netbsd",
                 "openbsd", "plan9", "solaris", "wasip1", "windows")


def build_ok(path, src, tags=("linux", "amd64", "unix", "cgo", "gc")):
    """Whether a file is in the build for GOOS=linux GOARCH=amd64 (plus tags): its //go:build line
    (&&, ||, !, parentheses) and its _GOOS / _GOARCH file-name suffixes."""
    base = os.path.basename(path)[:-3]
    parts = base.split("_")
    for p_ in parts[1:]:
        if p_ in GOOS_SUFFIXES and p_ != "linux":
            return False
    m = re.search(r"^//go:build (.+)$", src, re.M)
    if not m:
        return True
    expr = m.group(1).strip()
    toks = re.findall(r"&&|\|\||!|\(|\)|[\w.]+", expr)
    py = []
    for t in toks:
        py.append({"&&": " and ", "||": " or ", "!": " not ", "(": "(", ")": ")"}.get(t) or
                  (" True " if (t in tags or t.startswith("go1.")) else " False "))
    try:
        return bool(eval("".join(py), {"__builtins__": {}}))
    except SyntaxError:
        return True


def duplicate_decls(uni, pkg, files):
    """Package-level names declared more than once among the given files' sites."""
    base = {os.path.basename(f) for f in files}
    out = []
    for (p, name), sites in uni.decl_sites.items():
        own = [s for s in sites if s.split(":")[0] in base]
        if p == pkg and len(sites) > 1 and own:
            out.append((name, sites))
    return out
