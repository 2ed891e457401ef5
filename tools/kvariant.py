"""Build kernel variants for tools/kbench.hip: copy a product kernel out of aa_kernels.hip, rename it
kv_<name><MODE>, apply text edits guarded by MODE, and register launch names "<name>_m<MODE>".
usage: python tools/kvariant.py <spec.py>   (spec defines KERNEL, NAME, EDITS=[(old, new)], MODES, LAUNCH)"""
import re
import sys

ROOT = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))


def main():
    spec = {}
    exec(open(sys.argv[1]).read(), spec)
    src = open(f"{ROOT}/adaptive_amd/csrc/aa_kernels.hip").read()
    a = src.index(spec["KERNEL"])
    b = src.index("\n}\n", a) + 3
    k = src[a:b]
    k = re.sub(r"^template <[^>]*>\n", "", k)
    k = re.sub(r"void (k_\w+)\(", "void kv_" + spec["NAME"] + "(", k, count=1)
    k = spec.get("PREFIX", "template <int MODE>\n") + k
    for old, new in spec["EDITS"]:
        assert old in k, old
        k = k.replace(old, new)
    h = open(f"{ROOT}/tools/kbench.hip").read()
    h = re.sub(r"namespace aa \{\n// VARIANTS BEGIN.*?// VARIANTS END\n\}  // namespace aa\n\n", "", h, flags=re.S)
    h = re.sub(r"    // VARIANT LAUNCH BEGIN.*?    // VARIANT LAUNCH END\n", "", h, flags=re.S)
    marker = 'extern "C" int kb_time('
    h = h.replace(marker, "namespace aa {\n// VARIANTS BEGIN\n" + k + "// VARIANTS END\n}  // namespace aa\n\n" + marker, 1)
    launch = "    // VARIANT LAUNCH BEGIN\n"
    for m in spec["MODES"]:
        launch += (f'    }} else if (!strcmp(which, "{spec["NAME"]}_m{m}")) {{\n'
                   f'      auto kern = kv_{spec["NAME"]}<{m}>;\n' + spec["LAUNCH"] + "\n")
    launch += "    // VARIANT LAUNCH END\n"
    h = h.replace("    } else {\n      return false;", launch + "    } else {\n      return false;", 1)
    open(f"{ROOT}/tools/kbench.hip", "w").write(h)


if __name__ == "__main__":
    main()
