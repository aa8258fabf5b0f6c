"""The indexing guard (ECDNA_REP_ERR_INTERNAL, ABI v11) under fault injection (development tool). Needs a library
built with -DECDNA_INJECT_EMPTY_NPLUS (EXTRA=-DECDNA_INJECT_EMPTY_NPLUS bash tools/ab_build.sh WORKTREE inject),
selected with ECDNA_SSA_LIB: that build turns every event of a replicate with no N+ cell into an N+ event (DeathNPlus
under birth-death, ProliferateNPlus under pure birth) in the row stepper and in the bin stepper's runtime-flags
instances. Replicates start from N- cells only ({0: 10}); each must stop at its first event with error 5 and
stop reason Error, and the run must finish without a memory fault (without the guard the death wraps n+ and
indexes off the row). Usage: ECDNA_SSA_LIB=... python tools/inject_check.py"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ecdna-evo_amd"))
from ecdna_evo_amd import abi, engine  # noqa: E402


def main():
    ok = True
    for name, proc, flags in (("rows, birth-death", abi.BIRTH_DEATH, abi.FLAG_EVENT_HASH),
                              ("rows, pure birth", abi.PURE_BIRTH, abi.FLAG_EVENT_HASH),
                              ("bins K=64, birth-death, TF=1", abi.BIRTH_DEATH, abi.FLAG_BIN_STORE | abi.FLAG_EVENT_HASH),
                              ("bins K=32, birth-death, f32 time", abi.BIRTH_DEATH, abi.FLAG_BIN_STORE | abi.FLAG_TIME_F32),
                              ("bins K=64, pure birth, TF=1", abi.PURE_BIRTH, abi.FLAG_BIN_STORE | abi.FLAG_EVENT_HASH)):
        spec = abi.RunSpec(process=proc, rates=((1.0, 1.0, 0.3, 0.3) if proc else (1.0, 1.0, 0.0, 0.0),),
                           n_replicates=4096, init={0: 10}, max_cells=1000, flags=flags,
                           bin_kmax=32 if "K=32" in name else 64, seed=7)
        s = engine.run(spec).summaries
        good = bool((s["error"] == abi.REP_ERR_INTERNAL).all() and (s["stop_reason"] == abi.STOP_ERROR).all()
                    and (s["iters"] == 0).all() and (s["nminus"] == 10).all() and (s["nplus"] == 0).all())
        ok &= good
        print(json.dumps({"case": name, "replicates": len(s), "errors": sorted(set(s["error"].tolist())),
                          "stop_reasons": sorted(set(s["stop_reason"].tolist())), "max_iters": int(s["iters"].max()),
                          "ok": good}), flush=True)
    print(json.dumps({"all_ok": ok}))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
