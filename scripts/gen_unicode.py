"""Generate the Unicode class tables the regex compiler (fluvio_amd/csrc) and the
oracle's Pike VM (oracle/) share: General_Category ranges and the Perl \\w set
of regex-syntax (Alphabetic + M + Nd + Pc + Join_Control), from this image's
Python unicodedata.  The reference's regex crate carries Unicode 14
(regex-filter: regex-syntax 0.6.27) / 15 (examples: 0.7.1) tables, neither of
which is in the image: the code points whose General_Category differs between
unicodedata and the regex module's newer UCD (fsg_u_newer) make a
table-dependent pattern FSG_E_UNSUPPORTED.  Usage: python scripts/gen_unicode.py"""
import os
import sys
import unicodedata

CATS = ["Lu", "Ll", "Lt", "Lm", "Lo", "Mn", "Mc", "Me", "Nd", "Nl", "No", "Pc", "Pd", "Ps", "Pe", "Pi", "Pf", "Po",
        "Sm", "Sc", "Sk", "So", "Zs", "Zl", "Zp", "Cc", "Cf", "Cs", "Co", "Cn"]
# Other_Alphabetic code points outside M (PropList.txt): circled / squared Latin letters (So)
OALPHA_NON_M = [(0x24B6, 0x24E9), (0x1F130, 0x1F149), (0x1F150, 0x1F169), (0x1F170, 0x1F189)]


def ranges(pred):
    out, lo = [], None
    for c in range(0x110000):
        if pred(c):
            if lo is None:
                lo = c
        elif lo is not None:
            out.append((lo, c - 1))
            lo = None
    if lo is not None:
        out.append((lo, 0x10FFFF))
    return out


# regex-syntax's binary properties (property_bool.rs: PropList, DerivedCoreProperties,
# emoji-data) with their PropertyAliases.txt names; Changes_When_NFKC_Casefolded is
# left out (the Python regex module has no table for it: \p{CWKCF} stays unsupported)
BOOLS = [("ASCII_Hex_Digit", "AHex"), ("Alphabetic", "Alpha"), ("Bidi_Control", "Bidi_C"),
         ("Bidi_Mirrored", "Bidi_M"), ("Case_Ignorable", "CI"), ("Cased",), ("Changes_When_Casefolded", "CWCF"),
         ("Changes_When_Casemapped", "CWCM"), ("Changes_When_Lowercased", "CWL"), ("Changes_When_Titlecased", "CWT"),
         ("Changes_When_Uppercased", "CWU"), ("Dash",), ("Default_Ignorable_Code_Point", "DI"), ("Deprecated", "Dep"),
         ("Diacritic", "Dia"), ("Emoji",), ("Emoji_Component", "EComp"), ("Emoji_Modifier", "EMod"),
         ("Emoji_Modifier_Base", "EBase"), ("Emoji_Presentation", "EPres"), ("Extended_Pictographic", "ExtPict"),
         ("Extender", "Ext"), ("Grapheme_Base", "Gr_Base"), ("Grapheme_Extend", "Gr_Ext"), ("Grapheme_Link", "Gr_Link"),
         ("Hex_Digit", "Hex"), ("Hyphen",), ("IDS_Binary_Operator", "IDSB"), ("IDS_Trinary_Operator", "IDST"),
         ("ID_Continue", "IDC"), ("ID_Start", "IDS"), ("Ideographic", "Ideo"), ("Join_Control", "Join_C"),
         ("Logical_Order_Exception", "LOE"), ("Lowercase", "Lower"), ("Math",), ("Noncharacter_Code_Point", "NChar"),
         ("Other_Alphabetic", "OAlpha"), ("Other_Default_Ignorable_Code_Point", "ODI"),
         ("Other_Grapheme_Extend", "OGr_Ext"), ("Other_ID_Continue", "OIDC"), ("Other_ID_Start", "OIDS"),
         ("Other_Lowercase", "OLower"), ("Other_Math", "OMath"), ("Other_Uppercase", "OUpper"),
         ("Pattern_Syntax", "Pat_Syn"), ("Pattern_White_Space", "Pat_WS"), ("Prepended_Concatenation_Mark", "PCM"),
         ("Quotation_Mark", "QMark"), ("Radical",), ("Regional_Indicator", "RI"), ("Sentence_Terminal", "STerm"),
         ("Soft_Dotted", "SD"), ("Terminal_Punctuation", "Term"), ("Unified_Ideograph", "UIdeo"),
         ("Uppercase", "Upper"), ("Variation_Selector", "VS"), ("White_Space", "WSpace", "space"),
         ("XID_Continue", "XIDC"), ("XID_Start", "XIDS")]
# scripts the reference's Unicode 15 tables do not have (added in Unicode 16 / 17)
NEW_SCRIPTS = {"GARAY", "GURUNGKHEMA", "KIRATRAI", "OLONAL", "SUNUWAR", "TODHRI", "TULUTIGALARI", "BERIAERFE",
               "SIDETIC", "TAIYO", "TOLONGSIKI"}


def norm(name):
    return "".join(ch for ch in name.lower() if ch not in " _-")


def collapse(cps):
    out = []
    for c in cps:
        if out and out[-1][1] + 1 == c:
            out[-1][1] = c
        else:
            out.append([c, c])
    return [tuple(r) for r in out]


def props_and_folds():
    """Binary properties and Script / Script_Extensions values from the Python
    regex module (its UCD is newer than the reference's Unicode 15: code points
    assigned since differ, parity unpinned for them); simple case folding from
    this Python's str case mappings (Unicode 13)."""
    import regex
    import regex._regex_core as rc
    allc = "".join(chr(c) for c in range(0x110000))

    def cps_of(pat):
        return collapse(m.start() for m in regex.finditer(pat, allc))

    lines, sets, names = [], [], []
    gc_names = set()
    for i, k in enumerate(CATS):
        gc_names.add(k.lower())
    for b in BOOLS:
        rs = cps_of(r"\p{%s}" % b[0])
        idx = len(sets)
        sets.append(("b_" + b[0], rs))
        for a in b:
            n = norm(a)
            assert n not in gc_names or n == "space", n
            names.append((n, 1, idx))
    by_id = {}
    for nm, i in rc.PROPERTIES["SCRIPT"][1].items():
        by_id.setdefault(i, []).append(nm)
    for i, nms in sorted(by_id.items()):
        if any(n in NEW_SCRIPTS for n in nms):
            continue
        canon = max(nms, key=len)
        sc = cps_of(r"\p{Script=%s}" % canon)
        scx = cps_of(r"\p{Script_Extensions=%s}" % canon)
        si = len(sets)
        sets.append(("sc_" + canon, sc))
        sets.append(("scx_" + canon, scx))
        for n in nms:
            names.append((n.lower(), 2, si))
            names.append((n.lower(), 3, si + 1))
    # Grapheme_Cluster_Break / Word_Break / Sentence_Break values (gcb= / wb= /
    # sb=; regex-syntax's property_values; the value sets are Unicode 15's)
    for kind, (prop, short) in enumerate([("GRAPHEMECLUSTERBREAK", "gcb"), ("WORDBREAK", "wb"),
                                          ("SENTENCEBREAK", "sb")], start=4):
        by_id = {}
        for nm, i in rc.PROPERTIES[prop][1].items():
            by_id.setdefault(i, []).append(nm)
        for i, nms in sorted(by_id.items()):
            canon = max(nms, key=len)
            si = len(sets)
            sets.append(("%s_%s" % (short, canon), cps_of(r"\p{%s=%s}" % (prop, canon))))
            for n in nms:
                names.append((n.lower(), kind, si))
    for nm, rs in sets:
        lines.append("static const fsg_urange fsg_u_%s[] = {%s};" % (nm, ", ".join("{0x%X, 0x%X}" % r for r in rs) or "{1, 0}"))
    lines.append("static const fsg_urange* const fsg_u_psets[] = {%s};" % ", ".join("fsg_u_" + nm for nm, _ in sets))
    lines.append("static const uint32_t fsg_u_psets_n[] = {%s};" % ", ".join(str(len(rs)) for _, rs in sets))
    names.sort()
    lines.append("/* normalized name, kind (1 binary property, 2 Script value, 3 Script_Extensions value, 4 / 5 / 6 "
                 "Grapheme_Cluster_Break / Word_Break / Sentence_Break value), set */")
    lines.append("static const struct { const char *n; int k, s; } fsg_u_pnames[] = {" +
                 ", ".join('{"%s", %d, %d}' % t for t in names) + "};")
    lines.append("""/* a normalized \\p{..} name that is not a General_Category value: a binary
 * property, a Script value (bare or sc= / script=), a Script_Extensions value
 * (scx= / scriptextensions=) or a gcb= / wb= / sb= value, in regex-syntax's
 * order; 1 found, 0 unknown */
static int fsg_u_lookup(const char *name, const fsg_urange **r, uint32_t *n) {
  const char *eq = strchr(name, '=');
  int want = 0;
  const char *v = name;
  if (eq) {
    size_t pl = (size_t)(eq - name);
    if ((pl == 2 && !strncmp(name, "sc", 2)) || (pl == 6 && !strncmp(name, "script", 6))) want = 2;
    else if ((pl == 3 && !strncmp(name, "scx", 3)) || (pl == 16 && !strncmp(name, "scriptextensions", 16))) want = 3;
    else if ((pl == 3 && !strncmp(name, "gcb", 3)) || (pl == 20 && !strncmp(name, "graphemeclusterbreak", 20))) want = 4;
    else if ((pl == 2 && !strncmp(name, "wb", 2)) || (pl == 9 && !strncmp(name, "wordbreak", 9))) want = 5;
    else if ((pl == 2 && !strncmp(name, "sb", 2)) || (pl == 13 && !strncmp(name, "sentencebreak", 13))) want = 6;
    else return 0;
    v = eq + 1;
  } else if (!strcmp(name, "cf") || !strcmp(name, "sc") || !strcmp(name, "lc")) {
    return 0;
  }
  for (int pass = eq ? want : 1; pass <= (eq ? want : 2); pass++)
    for (size_t i = 0; i < sizeof fsg_u_pnames / sizeof fsg_u_pnames[0]; i++)
      if (fsg_u_pnames[i].k == pass && !strcmp(fsg_u_pnames[i].n, v)) {
        *r = fsg_u_psets[fsg_u_pnames[i].s];
        *n = fsg_u_psets_n[fsg_u_pnames[i].s];
        return 1;
      }
  return 0;
}""")
    # simple case folding (CaseFolding.txt statuses C + S, as ucd-generate builds
    # regex-syntax's table): a code point's simple fold is its casefold() when
    # that is one character (status C), else its lowercase when that is one
    # character (the S entry of an F code point: U+1E9E -> U+00DF, U+1F88 ->
    # U+1F80), else itself; the orbits are the classes of equal folds (Turkic T
    # entries stay out: U+0131 and U+0130 have none)
    def sfold(c):
        ch = chr(c)
        f = ch.casefold()
        if len(f) == 1:
            return ord(f)
        lo = ch.lower()
        return ord(lo) if len(lo) == 1 else c
    groups = {}
    for c in range(0x110000):
        if 0xD800 <= c <= 0xDFFF:
            continue
        groups.setdefault(sfold(c), set()).add(c)
    orbits = []
    for k, mem in groups.items():
        mem.add(k)
        if len(mem) > 1:
            orbits.append(sorted(mem))
    orbits.sort()
    cp_orb = []
    for oi, mem in enumerate(orbits):
        for c in mem:
            cp_orb.append((c, oi))
    cp_orb.sort()
    offs, flat = [], []
    for mem in orbits:
        offs.append(len(flat))
        flat += mem
    offs.append(len(flat))
    lines.append("/* simple case folding: code points with case-fold equivalents, their orbit, the orbits' members */")
    lines.append("static const uint32_t fsg_u_fold_cp[] = {%s};" % ", ".join("0x%X" % c for c, _ in cp_orb))
    lines.append("static const uint16_t fsg_u_fold_orb[] = {%s};" % ", ".join(str(o) for _, o in cp_orb))
    lines.append("static const uint16_t fsg_u_orb_off[] = {%s};" % ", ".join(str(o) for o in offs))
    lines.append("static const uint32_t fsg_u_orb_mem[] = {%s};" % ", ".join("0x%X" % c for c in flat))
    lines.append("static const uint32_t fsg_u_fold_n = %d;" % len(cp_orb))
    lines.append("""/* every case-fold equivalent of the code points in [lo, hi] (their orbits' members) */
static void fsg_u_fold_range(uint32_t lo, uint32_t hi, void (*add)(void *, uint32_t), void *ctx) {
  uint32_t a = 0, b = fsg_u_fold_n;
  while (a < b) {
    uint32_t m = (a + b) / 2;
    if (fsg_u_fold_cp[m] < lo) a = m + 1; else b = m;
  }
  for (uint32_t i = a; i < fsg_u_fold_n && fsg_u_fold_cp[i] <= hi; i++) {
    uint32_t o = fsg_u_fold_orb[i];
    for (uint32_t j = fsg_u_orb_off[o]; j < fsg_u_orb_off[o + 1]; j++) add(ctx, fsg_u_orb_mem[j]);
  }
}""")
    print(f"{len(sets)} property sets ({sum(len(r) for _, r in sets)} ranges), {len(orbits)} fold orbits", file=sys.stderr)
    return lines


def regex_version():
    import regex
    return regex.__version__


def main():
    cat = [unicodedata.category(chr(c)) for c in range(0x110000)]
    oalpha = set()
    for lo, hi in OALPHA_NON_M:
        oalpha.update(range(lo, hi + 1))
    tabs = {k: ranges(lambda c, k=k: cat[c] == k) for k in CATS}
    word = ranges(lambda c: cat[c][0] in "LM" or cat[c] in ("Nd", "Nl", "Pc") or c in (0x200C, 0x200D) or c in oalpha)
    lines = ["/* generated by scripts/gen_unicode.py from Python unicodedata %s: General_Category" % unicodedata.unidata_version,
             " * ranges and regex-syntax's Perl \\\\w (Alphabetic + M + Nd + Pc + Join_Control); binary properties,",
             " * scripts from the Python regex module, simple case folding from str case mappings.  Do not edit. */",
             "#pragma once", "#include <stdint.h>", "#include <string.h>", "#include <stddef.h>",
             "typedef struct { uint32_t lo, hi; } fsg_urange;",
             "#define FSG_UNICODE_VERSION \"%s\"" % unicodedata.unidata_version,
             "/* binary properties, scripts, break properties: the Python regex module %s (Unicode 17 by its"
             " assigned-character count); the reference: regex-syntax 0.6.27 (Unicode 14, regex-filter) and"
             " 0.7.1 (Unicode 15, filter_regex) */" % regex_version(),
             "#define FSG_UNICODE_PROPS_SOURCE \"regex %s\"" % regex_version(),
             "#define FSG_UNICODE_REFERENCE \"14.0 (regex-syntax 0.6.27) / 15.0 (regex-syntax 0.7.1)\""]
    def arr(name, rs):
        body = ", ".join("{0x%X, 0x%X}" % r for r in rs)
        lines.append("static const fsg_urange fsg_u_%s[] = {%s};" % (name, body))
    for k in CATS:
        arr(k, tabs[k])
    arr("word", word)
    # Rust's str Debug (core fmt, toolchain 1.75): a char is written as \u{..}
    # when it is not printable (printable.py: General_Category Cc Cf Cs Co Cn Zl
    # Zp Zs, the space excepted) or Grapheme_Extend (escape_grapheme_extended);
    # Grapheme_Extend from the Python regex module, on code points unicodedata
    # assigns (later ones are Cn here: parity unpinned for them)
    import regex
    gext = regex.compile(r"\p{Grapheme_Extend}")
    dbg = ranges(lambda c: (cat[c] in ("Cc", "Cf", "Cs", "Co", "Cn", "Zl", "Zp", "Zs") and c != 0x20) or
                 (cat[c] != "Cn" and gext.match(chr(c)) is not None))
    arr("dbgesc", dbg)
    lines.append("static const uint32_t fsg_u_dbgesc_n = %d;" % len(dbg))
    lines.append("/* 1: Rust's str Debug writes code point cp as \\u{..} (fsg_u_dbgesc) */")
    lines.append("static int fsg_u_dbg_escaped(uint32_t cp) {")
    lines.append("  uint32_t lo = 0, hi = fsg_u_dbgesc_n;")
    lines.append("  while (lo < hi) {")
    lines.append("    const uint32_t m = (lo + hi) / 2;")
    lines.append("    if (cp < fsg_u_dbgesc[m].lo) hi = m;")
    lines.append("    else if (cp > fsg_u_dbgesc[m].hi) lo = m + 1;")
    lines.append("    else return 1;")
    lines.append("  }")
    lines.append("  return 0;")
    lines.append("}")
    # version-uncertain code points: General_Category differs between this
    # image's unicodedata and the regex module's UCD (every code point assigned
    # after unicodedata's version, plus gc changes such as U+0295 Ll -> Lo).
    # regex-filter emulates regex-syntax 0.6.27 (Unicode 14), filter_regex
    # regex-syntax 0.7.1 (Unicode 15); neither version's tables are in the
    # image, so a table-dependent pattern meeting one of these code points is
    # FSG_E_UNSUPPORTED (device and oracle alike) rather than a guess
    allc = "".join(chr(c) for c in range(0x110000))
    rgc = ["Cn"] * 0x110000
    for k in CATS:
        for m in regex.finditer(r"\p{gc=%s}" % k, allc):
            rgc[m.start()] = k
    newer = ranges(lambda c: rgc[c] != cat[c])
    arr("newer", newer)
    lines.append("static const uint32_t fsg_u_newer_n = %d;" % len(newer))
    lines.append("/* 1: code point cp is version-uncertain (fsg_u_newer) */")
    lines.append("static int fsg_u_is_newer(uint32_t cp) {")
    lines.append("  uint32_t lo = 0, hi = fsg_u_newer_n;")
    lines.append("  while (lo < hi) {")
    lines.append("    const uint32_t m = (lo + hi) / 2;")
    lines.append("    if (cp < fsg_u_newer[m].lo) hi = m;")
    lines.append("    else if (cp > fsg_u_newer[m].hi) lo = m + 1;")
    lines.append("    else return 1;")
    lines.append("  }")
    lines.append("  return 0;")
    lines.append("}")
    lines.append("""/* a normalized \\p{..} name neither fsg_u_property nor fsg_u_lookup resolves,
 * as regex-syntax's unicode.rs canonicalizes it: 1 a property it supports that
 * is not restated here (Age values, Changes_When_NFKC_Casefolded:
 * FSG_E_UNSUPPORTED), 2 a known enumerated property with an unknown value
 * ("Unicode property value not found"), 3 anything else, a Unicode 16+ script
 * included ("Unicode property not found") */
static int fsg_u_unresolved(const char *name) {
  static const char *const enumerated[] = {"gc", "generalcategory", "sc", "script", "scx", "scriptextensions",
                                           "gcb", "graphemeclusterbreak", "wb", "wordbreak", "sb", "sentencebreak"};
  const char *eq = strchr(name, '=');
  if (!eq) return (!strcmp(name, "cwkcf") || !strcmp(name, "changeswhennfkccasefolded")) ? 1 : 3;
  const size_t pl = (size_t)(eq - name);
  if (pl == 3 && !strncmp(name, "age", 3)) return 1;
  for (size_t i = 0; i < sizeof enumerated / sizeof enumerated[0]; i++)
    if (strlen(enumerated[i]) == pl && !strncmp(name, enumerated[i], pl)) return 2;
  return 3;
}""")
    lines.append("typedef struct { const char *name; const fsg_urange *r; uint32_t n; } fsg_ucat;")
    lines.append("static const fsg_ucat fsg_u_cats[] = {" + ", ".join(
        '{"%s", fsg_u_%s, %d}' % (k, k, len(tabs[k])) for k in CATS) + "};")
    lines.append("static const uint32_t fsg_u_ncats = %d;" % len(CATS))
    lines.append("static const uint32_t fsg_u_word_n = %d;" % len(word))
    # property names of \p{..} (UCD PropertyValueAliases for General_Category, plus
    # Any / ASCII / Assigned / White_Space), normalized as regex-syntax does
    # (ASCII lowercase, ' ', '_' and '-' removed)
    groups = {"l": "Lu Ll Lt Lm Lo", "lc": "Lu Ll Lt", "m": "Mn Mc Me", "n": "Nd Nl No", "p": "Pc Pd Ps Pe Pi Pf Po",
              "s": "Sm Sc Sk So", "z": "Zs Zl Zp", "c": "Cc Cf Cs Co Cn"}
    alias = {"letter": "l", "casedletter": "lc", "mark": "m", "combiningmark": "m", "number": "n",
             "punctuation": "p", "punct": "p", "symbol": "s", "separator": "z", "other": "c",
             "uppercaseletter": "lu", "lowercaseletter": "ll", "titlecaseletter": "lt", "modifierletter": "lm",
             "otherletter": "lo", "nonspacingmark": "mn", "spacingmark": "mc", "enclosingmark": "me",
             "decimalnumber": "nd", "digit": "nd", "letternumber": "nl", "othernumber": "no",
             "connectorpunctuation": "pc", "dashpunctuation": "pd", "openpunctuation": "ps",
             "closepunctuation": "pe", "initialpunctuation": "pi", "finalpunctuation": "pf",
             "otherpunctuation": "po", "mathsymbol": "sm", "currencysymbol": "sc", "modifiersymbol": "sk",
             "othersymbol": "so", "spaceseparator": "zs", "lineseparator": "zl", "paragraphseparator": "zp",
             "control": "cc", "cntrl": "cc", "format": "cf", "surrogate": "cs", "privateuse": "co",
             "unassigned": "cn"}
    masks = {}
    for i, k in enumerate(CATS):
        masks[k.lower()] = 1 << i
    for g, ks in groups.items():
        masks[g] = sum(1 << CATS.index(k) for k in ks.split())
    for a, t in alias.items():
        masks[a] = masks[t]
    masks["any"] = (1 << len(CATS)) - 1
    masks["assigned"] = masks["any"] & ~(1 << CATS.index("Cn"))
    entries = sorted(masks.items())
    lines.append("#define FSG_UPROP_ASCII (-2)")
    lines.append("#define FSG_UPROP_WSPACE (-3)")
    lines.append("/* a normalized \\p{..} name -> a mask of fsg_u_cats indices, FSG_UPROP_ASCII / _WSPACE, -1 unknown */")
    lines.append("static long fsg_u_property(const char *name) {")
    lines.append("  static const struct { const char *n; long m; } T[] = {" +
                 ", ".join('{"%s", %dL}' % (k, v) for k, v in entries) + "};")
    lines.append("  const char *nm = name;")
    lines.append('  if (!strncmp(nm, "gc=", 3)) nm += 3;')
    lines.append('  else if (!strncmp(nm, "generalcategory=", 16)) nm += 16;')
    lines.append('  if (!strcmp(nm, "ascii")) return FSG_UPROP_ASCII;')
    lines.append('  if (!strcmp(nm, "whitespace") || !strcmp(nm, "wspace") || !strcmp(nm, "space")) return FSG_UPROP_WSPACE;')
    lines.append("  for (size_t i = 0; i < sizeof T / sizeof T[0]; i++)")
    lines.append("    if (!strcmp(T[i].n, nm)) return T[i].m;")
    lines.append("  return -1;")
    lines.append("}")
    lines += props_and_folds()
    text = "\n".join(lines) + "\n"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for d in ("fluvio_amd/csrc", "oracle"):
        with open(os.path.join(root, d, "fsg_unicode.h"), "w") as f:
            f.write(text)
    print(f"{sum(len(v) for v in tabs.values())} category ranges, {len(word)} word ranges", file=sys.stderr)


if __name__ == "__main__":
    main()
