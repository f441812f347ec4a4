// The README Cornell box (SURVEY §8(d) C1/C2) as an editor-style scene script for sail_amd/js/cli.js:
//   node sail_amd/js/cli.js sail_amd/js/examples/cornell.js --spp 256 --png cornell.png --pfm cornell.pfm
scene = new Sail.Scene();
// ceiling light: a thin emissive cube
scene.add(new Sail.Cube([2.13, 5.487, 2.27], [3.43, 5.488, 3.32], new Sail.Matte(0.7),
  Sail.Color.createTexture([0, 0, 0]), [8, 8, 8]));
scene.add(new Sail.Cornellbox([0, 0, -7], [5.560, 5.488, 5.592]));
scene.add(new Sail.Sphere([2, 1.25, 2.70], 1.2, new Sail.Mirror(1.0), Sail.Color.WHITE));
scene.add(new Sail.Camera([2.78, 2.73, -6], [2.78, 2.73, 2.79]));
scene.filter = 'tonemapping';
