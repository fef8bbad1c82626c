"""The interior point's generated inline asm (csrc/osc_ipm_asm.hpp) is what tools/gen_ipm_asm.py
produces: nobody edits the header by hand, and a generator change is rebuilt into it (CPU only)."""
import importlib.util
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_osc_ipm_asm_matches_generator():
    spec = importlib.util.spec_from_file_location("gen_ipm_asm",
                                                  os.path.join(REPO, "tools", "gen_ipm_asm.py"))
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)
    with open(gen.OUT) as f:
        assert f.read() == gen.render()


def test_ldl_schedule_wait_slots_bounded():
    # the scheduler fills nearly every hazard wait with an FMA (DESIGN.md §5 "Issue slots")
    spec = importlib.util.spec_from_file_location("gen_ipm_asm",
                                                  os.path.join(REPO, "tools", "gen_ipm_asm.py"))
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)
    for n in (24, 32):
        ins, _ = gen.ldl(n)
        waits = sum(int(t.split()[1]) + 1 for t in ins if t.startswith("s_nop"))
        assert waits <= 40, (n, waits)
