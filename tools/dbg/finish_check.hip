// Diagnostic: bold_finish on device vs a host replica of the same loop.
#include "../../nremmodfc_amd/csrc/wc_signal.hip"
#include <vector>
int main() {
  wc_bold_cfg cfg; cfg.dt = 0.04; cfg.neq = 2000; cfg.n_total = 6000; cfg.dec = 1000;
  double b[5] = {0.00012544743505202416,0.0,-0.0002508948701040483,0.0,0.00012544743505202416}, a[5] = {1.0,-3.9609509668036016,5.883482227394972,-3.8841091195101143,0.9615778628317615}, zi[4] = {-0.00012544743168405392,-0.000125447445024419,0.00012544744489502245,0.00012544743181345855};
  for (int i = 0; i < 5; ++i) { cfg.b[i] = b[i]; cfg.a[i] = a[i]; } for (int i = 0; i < 4; ++i) cfg.zi[i] = zi[i];
  const int64_t C = 1; const BoldLayout L(C, 4, 1000);
  std::vector<double> st(L.total, 0.0);
  double zend[4] = {-1.91709774e-07, 5.60857302e-07, -5.29137940e-07, 1.59990415e-07};
  double yzs[4] = {-8.067896010999195e-05, 0.00011468659284840595, 0.00020640665221173624, 3.6106456123367825e-06};
  double u[4][4] = {{-7.83742728e-05, 2.34383732e-04, -2.33588194e-04, 7.75788179e-05}, {0.00011579, -0.00034186, 0.00033631, -0.00011025},
                    {0.00020378, -0.00060609, 0.00060078, -0.00019847}, {3.18365113e-06, -9.80475595e-06, 1.01020816e-05, -3.48090278e-06}};
  for (int k = 0; k < 4; ++k) st[L.zend + k] = zend[k];
  for (int m = 0; m < 4; ++m) { st[L.yzs + m] = yzs[m]; for (int k = 0; k < 4; ++k) st[L.u + m * 4 + k] = u[m][k]; }
  double *dst, *dout; hipMalloc(&dst, st.size() * 8); hipMalloc(&dout, 4 * 8);
  hipMemcpy(dst, st.data(), st.size() * 8, hipMemcpyHostToDevice);
  int rc = wc_bold_finish(&cfg, C, dst, dout, nullptr); hipDeviceSynchronize();
  double o[4]; hipMemcpy(o, dout, 32, hipMemcpyDeviceToHost);
  printf("rc %d dev: %g %g %g %g\n", rc, o[0], o[1], o[2], o[3]);
  // host replica
  cld lam[4], Vi[16]; poles(cfg.a, lam); modal_inverse(cfg.a, lam, Vi);
  cdd fVi[16], lamL[4], lamL1[4];
  for (int i = 0; i < 16; ++i) fVi[i] = to_cdd(Vi[i]);
  for (int i = 0; i < 4; ++i) { lamL[i] = to_cdd(cpow_int(lam[i], 1000)); lamL1[i] = to_cdd(cpow_int(lam[i], 999)); }
  cdd w[4];
  for (int i = 0; i < 4; ++i) { cdd acc = {{0,0},{0,0}}; for (int k = 0; k < 4; ++k) acc = cdd_add(acc, cdd_mul_d(fVi[i*4+k], zend[k])); w[i] = acc; }
  for (int m = 3; m >= 0; --m) {
    dd y = {yzs[m], 0.0};
    for (int i = 0; i < 4; ++i) y = dd_add(y, cdd_mul(lamL1[i], w[i]).re);
    printf("host m=%d out=%g\n", m, y.hi + y.lo);
    for (int i = 0; i < 4; ++i) { cdd acc = cdd_mul(lamL[i], w[i]); for (int k = 0; k < 4; ++k) acc = cdd_add(acc, cdd_mul_d(fVi[i*4+k], u[m][k])); w[i] = acc; }
  }
  return 0;
}
