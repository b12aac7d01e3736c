"""Minimal SGF (FF[1]-FF[4]) parser.

The reference depends on the external ``sgf`` 0.5 package (util.py:4, game_converter.py:9), which
is not available here, so this is our own recursive-descent parser. It exposes just what the
reference pipeline consumes: a collection of games, each with a ``root`` node and the ``rest`` of
its *main line* (first variation at every branch), every node carrying a ``properties`` dict of
``ident -> [values]``.
"""


class SGFParseError(Exception):
    """Raised for malformed SGF (the reference's ``sgf.ParseException``)."""


class Node(object):
    __slots__ = ("properties",)

    def __init__(self, properties):
        self.properties = properties

    def __repr__(self):
        return "Node(%r)" % (self.properties,)


class GameTree(object):
    __slots__ = ("nodes", "variations")

    def __init__(self, nodes, variations):
        self.nodes = nodes
        self.variations = variations

    @property
    def root(self):
        return self.nodes[0]

    @property
    def rest(self):
        """Main-line nodes after the root (None when the game has no moves)."""
        out = []
        tree = self
        first = True
        while tree is not None:
            out.extend(tree.nodes[1:] if first else tree.nodes)
            first = False
            tree = tree.variations[0] if tree.variations else None
        return out if out else None


class _Parser(object):
    def __init__(self, text):
        self.s = text
        self.i = 0
        self.n = len(text)

    def _ws(self):
        s, n = self.s, self.n
        while self.i < n and s[self.i] in " \t\r\n\x0b\x0c":
            self.i += 1

    def _expect(self, ch):
        self._ws()
        if self.i >= self.n or self.s[self.i] != ch:
            got = self.s[self.i] if self.i < self.n else "EOF"
            raise SGFParseError("expected %r at offset %d, got %r" % (ch, self.i, got))
        self.i += 1

    def collection(self):
        games = []
        self._ws()
        while self.i < self.n:
            if self.s[self.i] != "(":
                # tolerate trailing garbage after the last game
                if games:
                    break
                raise SGFParseError("SGF must start with '('")
            games.append(self.gametree())
            self._ws()
        if not games:
            raise SGFParseError("empty SGF collection")
        return games

    def gametree(self):
        self._expect("(")
        nodes = []
        self._ws()
        while self.i < self.n and self.s[self.i] == ";":
            self.i += 1
            nodes.append(self.node())
            self._ws()
        if not nodes:
            raise SGFParseError("game tree without nodes at offset %d" % self.i)
        variations = []
        while self.i < self.n and self.s[self.i] == "(":
            variations.append(self.gametree())
            self._ws()
        self._expect(")")
        return GameTree(nodes, variations)

    def node(self):
        props = {}
        s = self.s
        while True:
            self._ws()
            if self.i >= self.n or not s[self.i].isalpha():
                break
            start = self.i
            while self.i < self.n and s[self.i].isalpha():
                self.i += 1
            ident = "".join(c for c in s[start:self.i] if c.isupper())  # FF[3] lowercase letters
            values = []
            self._ws()
            while self.i < self.n and s[self.i] == "[":
                values.append(self.value())
                self._ws()
            if not values:
                raise SGFParseError("property %s without value" % ident)
            props.setdefault(ident, []).extend(values)
        return Node(props)

    def value(self):
        self.i += 1  # '['
        s = self.s
        out = []
        while True:
            if self.i >= self.n:
                raise SGFParseError("unterminated property value")
            c = s[self.i]
            if c == "\\":
                self.i += 1
                if self.i < self.n:
                    if s[self.i] == "\n":  # soft line break
                        pass
                    else:
                        out.append(s[self.i])
                self.i += 1
                continue
            if c == "]":
                self.i += 1
                return "".join(out)
            out.append(c)
            self.i += 1


def parse(text):
    """Parse an SGF string into a list of GameTree objects."""
    if isinstance(text, bytes):
        text = text.decode("utf-8", errors="replace")
    return _Parser(text).collection()
