"""Drop-in for the reference's ``src/convert_mgf_cluster.py`` MGF route: MaxQuant
msms.txt + MaRaCluster clusters + an MGF -> a clustered MGF whose titles follow
the cluster-title convention (``<cluster>;mzspec:<PXD>:<raw>:scan:<n>[:<seq>/<z>]``)
that binning.py / best_spectrum.py read.

* :func:`buid_usi_accession` (convert_mgf_cluster.py:14-18, the name keeps the
  reference's spelling)
* :func:`read_peptides` (:21-30): scan -> sequence (column 8 without its first and
  last character, MaxQuant's ``_SEQ_``); later rows overwrite earlier ones
* :func:`read_clusters` (:33-44): scan -> ``cluster-<k>``, k starting at 1 and
  advancing at every blank line
* :func:`convert_mq_mracluster_mgf` (:47-79): for every clustered scan in TSV
  order, every MGF spectrum whose title ends with ``scan=<n>`` is retitled and
  appended to the output.  The reference scans the whole spectrum list per
  scan (O(clusters x spectra)); here one title index gives the same matches in
  the same order.

The mzML route (``convert-mq-marcluster-mzml``, :82-124) stores OpenMS mzML
through pyopenms and stays out of scope (OpenMS I/O).  Host-side
data preparation -- no device work.
"""
from __future__ import annotations

import sys

from .mgf import iter_mgf, write_pyteomics_style


def buid_usi_accession(cluster_id, peptide_sequence, scan, px_accession, raw_name, charge):
    usi = cluster_id + ";" + "mzspec" + ":" + px_accession + ":" + raw_name + ":" + "scan:" + str(scan)
    if peptide_sequence is not None:
        usi = usi + ":" + peptide_sequence + "/" + str(charge)
    return usi


def read_peptides(mq_msms):
    peptides = {}
    with open(mq_msms) as fh:
        next(fh)  # header
        for line in fh:
            words = line.split("\t")
            peptides[int(words[1])] = words[7][1:-1]
    return peptides


def read_clusters(mrcluster_clusters):
    clusters = {}
    cluster_index = 1
    with open(mrcluster_clusters) as fh:
        for line in fh:
            if not line.strip():
                cluster_index += 1
            else:
                clusters[int(line.split("\t")[1])] = "cluster-" + str(cluster_index)
    return clusters


def _scan_suffix(title: str):
    i = title.rfind("scan=")
    return None if i < 0 else title[i + 5:]


def convert_mq_mracluster_mgf(mq_msms, mrcluster_clusters, mgf_file, output, px_accession, raw_name):
    """convert_mgf_cluster.py:47-79 (the ``convert-mq-marcluster`` command)."""
    if mq_msms is None or mrcluster_clusters is None or mgf_file is None:
        raise SystemExit("convert-mq-marcluster needs --mq_msms, --mrcluster_clusters and --mgf_file")
    spectra_list = list(iter_mgf(mgf_file))
    print("Number of Spectra: " + str(len(spectra_list)))
    peptides = read_peptides(mq_msms)
    print("Number of Peptides: " + str(len(peptides)))
    clusters = read_clusters(mrcluster_clusters)
    print("Number of Clusters: " + str(len(clusters)))
    by_suffix = {}
    for sp in spectra_list:
        by_suffix.setdefault(_scan_suffix(sp["params"]["title"]), []).append(sp)
    out = []
    for scan in clusters:
        print("scan: " + str(scan))
        for sp in by_suffix.get(str(scan), []):
            charge = int(sp["params"]["charge"][0])
            sp["params"]["title"] = buid_usi_accession(clusters[scan], peptides.get(scan), scan, px_accession,
                                                       raw_name, charge)
            out.append(sp)
    # the reference appends each spectrum to OUTPUT with pyteomics mgf.write
    write_pyteomics_style(out, output, file_mode="a")
    return out


def main(argv=None):
    import click

    @click.group(context_settings=dict(help_option_names=["-h", "--help"]))
    def cli():
        """Convert MaxQuant results and MaRaCluster clusters into a clustered MGF."""

    @cli.command("convert-mq-marcluster")
    @click.option("--mq_msms", "-p", help="Peptide information from MaxQuant")
    @click.option("--mrcluster_clusters", "-c", help="The information of the clusters from MaRCluster")
    @click.option("--mgf_file", "-s", help="The mgf with the corresponding spectra")
    @click.option("--output", "-o", help="Output mgf containing the cluster and the spectra information")
    @click.option("--px_accession", "-a", help="ProteomeXchange accession of the project")
    @click.option("--raw_name", "-r", help="Original name of the RAW file in proteomeXchange")
    def _mgf(mq_msms, mrcluster_clusters, mgf_file, output, px_accession, raw_name):
        convert_mq_mracluster_mgf(mq_msms, mrcluster_clusters, mgf_file, output, px_accession, raw_name)

    return cli.main(args=argv, standalone_mode=argv is None)


if __name__ == "__main__":
    sys.exit(main())
