// Metal, mirror, glass and textured matte spheres in a checkered room lit by an area light (SURVEY §8(d) C3).
scene = new Sail.Scene();
let matte = new Sail.Matte(0.7);
scene.add(new Sail.AreaLight(new Sail.Rectangle([2.13, 5.48, 2.27], [3.43, 5.48, 3.32], matte, Sail.Color.BLACK), [4, 4, 4]));
scene.add(new Sail.Cube([0, 0, -7], [5.56, 5.488, 5.592], matte, new Sail.Checkerboard(0.1, 0.01)));
scene.add(new Sail.Sphere([1.0, 0.8, 1.5], 0.8, new Sail.Metal(0, 0.01, 0.1), Sail.Color.WHITE));
scene.add(new Sail.Sphere([2.2, 0.8, 2.8], 0.8, new Sail.Mirror(1.0), Sail.Color.WHITE));
scene.add(new Sail.Sphere([3.4, 0.8, 1.5], 0.8, new Sail.Glass(1, 1, 1.5), Sail.Color.WHITE));
scene.add(new Sail.Sphere([4.6, 0.8, 2.8], 0.8, matte, new Sail.Checkerboard2([1, 1, 1], [0.2, 0.2, 0.2], 0.1)));
scene.add(new Sail.Camera([2.78, 2.73, -6], [2.78, 2.73, 2.79]));
scene.filter = 'gaussian';
scene.filter.addParam('r', 'vec2(2.0,2.0)');
scene.filter.addParam('alpha', '2.0');
