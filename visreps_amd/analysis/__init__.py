"""Mirror of visreps.analysis: rsa (RDM / RDM comparison / RSA) and alignment."""
