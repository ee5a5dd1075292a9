"""`python -m nldsc_amd ld ...` — the `nldsc ld` command (nldsc/__main__.py:35-97) on the GPU engine."""
import sys

import click

from . import __version__
from .core.logger import log

__header__ = (f"\n==============================================================\n"
              f"* Non-additive LD Score Regression (NLDSC) — MI355X engine v{__version__}\n"
              f"* LD-score compute path re-implemented for AMD Instinct MI355X (gfx950)\n"
              f"* Interface of bayarpark/nldsc `nldsc ld` (GPL-3.0)\n"
              f"==============================================================\n")


def handle_exception(func):
    """Same failure shape as the reference (nldsc/__main__.py:17-26)."""
    def handler(*args, **kwargs):
        display = kwargs.pop("display", None)
        try:
            return func(*args, **kwargs)
        except Exception as ex:  # noqa: BLE001
            log.critical(f"The program crashed with {ex.__class__.__name__}, what: {str(ex)}\n"
                         f"Use `--display` flag for traceback", exc_info=display)
            raise SystemExit()
    handler.__name__ = func.__name__
    handler.__doc__ = func.__doc__
    return handler


@click.group()
@click.version_option(version=__version__)
def main():
    click.echo(__header__)


@main.command("ld", help="Estimate additive and non-additive LD Scores")
@click.option("--bfile", help="Path prefix for PLINK .bed/.bim/.fam file or path to one of them; '@' in place of "
                               "the chromosome number runs every chromosome (then --out needs '@' too)", metavar="FILE",
              required=True)
@click.option("-o", "--out", help="Output path of the LD score table", metavar="FILE")
@click.option("-kb", "--ld-wind-kb", help="Window size in kilo-base pairs (kb)", metavar="W")
@click.option("-cm", "--ld-wind-cm", help="Window size in centi-morgans (cM)", metavar="W")
@click.option("-maf", "--maf-thr", help="Minor allele frequency threshold (lower bound)", metavar="F")
@click.option("-std", "--std-thr", help="Standard deviation threshold for regression residuals", metavar="F",
              default=1e-4)
@click.option("-rsq", "--rsq-thr", help="R-squared threshold for regression residual. It affects only dominant "
                                        "window sizes and, therefore, non-additive sample size (MD)", metavar="F")
@click.option("--extra", help="Include additional information to the .L2 file", is_flag=True, default=False)
@click.option("--write-m", help="Also write <out>.M with M and MD (as the h2 reader derives them)", is_flag=True,
              default=False)
@click.option("--strict-plink-order", help="Use PLINK sample order in the last .bed byte (the reference does not)",
              is_flag=True, default=False)
@click.option("--additive-only", help="Skip the dominance terms (L2D = NaN)", is_flag=True, default=False)
@click.option("--device", help="HIP device ordinal", type=int, default=None)
@click.option("--quiet", help="No progress lines on stderr", is_flag=True, default=False)
@click.option("--display", help="Display traceback", is_flag=True, default=False)
@handle_exception
def est_ld(bfile, out, ld_wind_kb, ld_wind_cm, maf_thr, std_thr, rsq_thr, extra, write_m, strict_plink_order,
           additive_only, device, quiet):
    if sum(map(bool, [ld_wind_kb, ld_wind_cm])) != 1:
        raise RuntimeError("Please, specify exactly one --ld-wind option")
    elif ld_wind_kb:
        wind_metric, ld_wind = "kbp", ld_wind_kb
    else:
        wind_metric, ld_wind = "cm", ld_wind_cm
    from .ldscore import _ldscore, estimate_lds
    flags = (_ldscore.FLAG_STRICT_PLINK_ORDER if strict_plink_order else 0) | \
            (_ldscore.FLAG_ADDITIVE_ONLY if additive_only else 0)
    if "@" in bfile:  # whole genome: one output per chromosome, chromosomes spread over GPUs
        from .ldscore.genome import estimate_lds_genome
        estimate_lds_genome(bfile, ld_wind=ld_wind, wind_metric=wind_metric, maf_thr=maf_thr, std_thr=std_thr,
                            rsq_thr=rsq_thr, out=out, extra=extra, write_m=write_m, flags=flags, device=device,
                            progress=not quiet)
        return
    estimate_lds(bfile, ld_wind=ld_wind, wind_metric=wind_metric, maf_thr=maf_thr, std_thr=std_thr,
                 rsq_thr=rsq_thr, out=out, extra=extra, summary=True, write_m=write_m, flags=flags, device=device,
                 progress=not quiet)


@main.command("h2", help="(not part of this engine) heritability estimation")
def est_h2():
    raise SystemExit("`h2` is out of scope for nldsc_amd: run the reference's `nldsc h2` on the .L2 output.")


if __name__ == "__main__":
    sys.exit(main())
