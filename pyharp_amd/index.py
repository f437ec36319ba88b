"""Layout constants of the optics / flux tensors (mirror of src/index.h:12-18)."""

# optical variables: prop[..., IEX] layer optical thickness, [..., ISS]
# single-scattering albedo, [..., IPM:] phase moments chi_1..chi_nmom
IEX = 0
ISS = 1
IPM = 2

# flux variables: flux[..., IUP] upward, [..., IDN] downward (rfldir + rfldn)
IUP = 0
IDN = 1
